/* fd_vtile_main.c -- the served verify tile as a program of its own (fdgpu_tile): one process per verify
   tile, as the reference runs its tiles (src/disco/topo/fd_topo_run.c:66-153).  It joins the link and its
   GPU's verify service segment by their files and runs the tile's loop (fdgpu_link_run_tile): mcache polls,
   before_frag / during_frag / after_frags, HA dedup, publish.  It makes no GPU call; the service process
   that started it owns the GPU.

   usage: fdgpu_tile <link file> <service segment file> <tile> <cpu> [copy thread cpus ...] */

#include "../../include/fd_verify_gpu.h"

#include <stdio.h>
#include <stdlib.h>

int
main( int argc, char ** argv ) {
  if( argc < 5 ) { fprintf( stderr, "usage: %s <link> <service> <tile> <cpu> [copy cpus]\n", argv[0] ); return 2; }
  fdgpu_link_t * l = fdgpu_link_join( argv[1], 60. );
  if( !l ) { fprintf( stderr, "fdgpu_tile: cannot join link %s\n", argv[1] ); return 3; }
  int cc[ 8 ], ncc = 0;
  for( int i=5; i<argc && ncc<8; i++ ) cc[ ncc++ ] = atoi( argv[i] );
  int rc = fdgpu_link_run_tile( l, atoi( argv[3] ), argv[2], atoi( argv[4] ), cc, ncc );
  fdgpu_link_delete( l );
  return rc ? 1 : 0;
}
