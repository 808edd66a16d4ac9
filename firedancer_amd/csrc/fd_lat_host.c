/* Host build of the device half-size-scalar reduction (fd_gpu_lattice.h),
   for tests/test_lattice.py: the same source the hash kernel inlines. */
#include "fd_gpu_lattice.h"

int
fd_lat_halfsize_host( uint32_t c0[ 5 ], uint32_t c1m[ 5 ], int * c1neg, uint32_t const k[ 8 ] ) {
  return fd_lat_halfsize( c0, c1m, c1neg, k );
}
