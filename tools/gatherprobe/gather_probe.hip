// PCIe intake probe for the configs[4] stream: how fast can the GPU pull
// fd_txn_m_t records (1312 B, 64-B chunk aligned) out of registered host
// memory, the way fd_gather_kernel does, and what does a DMA copy of the
// same bytes reach.  Each variant runs alone on the device; times are HIP
// events around REPS launches.
//
//   gather64      one 64-lane group per record, arena + host out region (the engine today)
//   gather64_in   the same, arena only (no write-back to host)
//   gatherw_N     one wave per record, N records per 256-lane group, all loads issued before stores
//   dma           hipMemcpyAsync of the batch's contiguous bytes, host -> device
//   dma_d2h       hipMemcpyAsync device -> host of the same bytes
//   wr_host       kernel writes the bytes into host memory (the out-region write alone)
//
// build: hipcc --offload-arch=gfx950 -O3 -o tools/gatherprobe/gather_probe tools/gatherprobe/gather_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CHK(x) do { hipError_t e_ = (x); if( e_ != hipSuccess ) { fprintf( stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString( e_ ) ); exit( 1 ); } } while( 0 )

struct gat { unsigned long src; unsigned dst; unsigned sz; };

__global__ void __launch_bounds__( 64 ) g64( gat const * g, unsigned char * arena, unsigned char * out ) {
  gat r = g[ blockIdx.x ];
  uint4 const * s = (uint4 const *)r.src;
  uint4 * a = (uint4 *)( arena + r.dst );
  uint4 * o = (uint4 *)( out + r.dst );
  for( unsigned i=threadIdx.x; i<(r.sz>>4); i+=64u ) { uint4 v = s[i]; a[i] = v; if( out ) o[i] = v; }
}

// one wave per record, loads first (up to 2 x 16 B per lane covers 2048 B)
template<int W>
__global__ void __launch_bounds__( 64*W ) gw( gat const * g, unsigned n, unsigned char * arena, unsigned char * out ) {
  unsigned t = blockIdx.x * W + ( threadIdx.x >> 6 );
  unsigned l = threadIdx.x & 63u;
  if( t >= n ) return;
  gat r = g[ t ];
  uint4 const * s = (uint4 const *)r.src;
  unsigned q = r.sz >> 4;
  uint4 v0 = {0,0,0,0}, v1 = {0,0,0,0};
  if( l < q ) v0 = s[l];
  if( l + 64u < q ) v1 = s[l + 64u];
  uint4 * a = (uint4 *)( arena + r.dst );
  if( l < q ) a[l] = v0;
  if( l + 64u < q ) a[l+64u] = v1;
  if( out ) {
    uint4 * o = (uint4 *)( out + r.dst );
    if( l < q ) o[l] = v0;
    if( l + 64u < q ) o[l+64u] = v1;
  }
}

__global__ void wr( uint4 const * src, uint4 * dst, unsigned long n16 ) {
  for( unsigned long i = blockIdx.x * (unsigned long)blockDim.x + threadIdx.x; i < n16; i += (unsigned long)gridDim.x * blockDim.x )
    dst[i] = src[i];
}

int main( int argc, char ** argv ) {
  unsigned const REC = 1312, CHUNK = 64, STRIDE = ( REC + CHUNK - 1 ) / CHUNK * CHUNK;
  unsigned const REPS = 20;
  unsigned sizes[] = { 4096, 8192, 16384, 32768, 65536, 131072 };
  unsigned long maxn = 131072;
  unsigned char * hin; CHK( hipHostMalloc( (void **)&hin, maxn * STRIDE * 2, hipHostMallocMapped ) );
  unsigned char * hout; CHK( hipHostMalloc( (void **)&hout, maxn * STRIDE, hipHostMallocMapped ) );
  unsigned char * din, * dout;
  CHK( hipHostGetDevicePointer( (void **)&din, hin, 0 ) );
  CHK( hipHostGetDevicePointer( (void **)&dout, hout, 0 ) );
  memset( hin, 7, maxn * STRIDE * 2 ); memset( hout, 0, maxn * STRIDE );
  unsigned char * arena; CHK( hipMalloc( (void **)&arena, maxn * STRIDE ) );
  gat * dg; CHK( hipMalloc( (void **)&dg, maxn * sizeof(gat) ) );
  std::vector<gat> hg( maxn );
  srand( 1 );
  // records scattered over a 2x larger in region (the dcache holds more than one batch)
  for( unsigned long i=0; i<maxn; i++ ) {
    unsigned long c = ( i * 2 + ( rand() & 1 ) ) * STRIDE;
    hg[i].src = (unsigned long)( din + c ); hg[i].dst = (unsigned)( i * STRIDE ); hg[i].sz = REC;
  }
  CHK( hipMemcpy( dg, hg.data(), maxn * sizeof(gat), hipMemcpyHostToDevice ) );
  hipStream_t st; CHK( hipStreamCreateWithFlags( &st, hipStreamNonBlocking ) );
  hipEvent_t e0, e1; CHK( hipEventCreate( &e0 ) ); CHK( hipEventCreate( &e1 ) );
  printf( "%-12s %8s %10s %10s\n", "variant", "records", "us/launch", "GB/s(rec)" );
  char const * names[] = { "gather64", "gather64_in", "gatherw_1", "gatherw_4", "gatherw_4in", "dma", "dma_d2h", "wr_host" };
  for( unsigned si=0; si<sizeof(sizes)/sizeof(sizes[0]); si++ ) {
    unsigned n = sizes[si];
    for( int v=0; v<8; v++ ) {
      auto run = [&]() {
        switch( v ) {
        case 0: g64<<<n, 64, 0, st>>>( dg, arena, dout ); break;
        case 1: g64<<<n, 64, 0, st>>>( dg, arena, NULL ); break;
        case 2: gw<1><<<n, 64, 0, st>>>( dg, n, arena, dout ); break;
        case 3: gw<4><<<(n+3)/4, 256, 0, st>>>( dg, n, arena, dout ); break;
        case 4: gw<4><<<(n+3)/4, 256, 0, st>>>( dg, n, arena, NULL ); break;
        case 5: CHK( hipMemcpyAsync( arena, hin, (size_t)n * STRIDE, hipMemcpyHostToDevice, st ) ); break;
        case 6: CHK( hipMemcpyAsync( hout, arena, (size_t)n * STRIDE, hipMemcpyDeviceToHost, st ) ); break;
        case 7: wr<<<1024, 256, 0, st>>>( (uint4 const *)arena, (uint4 *)dout, (unsigned long)n * STRIDE / 16 ); break;
        }
      };
      run(); CHK( hipStreamSynchronize( st ) );
      CHK( hipEventRecord( e0, st ) );
      for( unsigned r=0; r<REPS; r++ ) run();
      CHK( hipEventRecord( e1, st ) );
      CHK( hipEventSynchronize( e1 ) );
      float ms; CHK( hipEventElapsedTime( &ms, e0, e1 ) );
      double us = ms * 1e3 / REPS;
      printf( "%-12s %8u %10.1f %10.2f\n", names[v], n, us, (double)n * REC / ( us * 1e3 ) );
    }
  }
  // check: the last gather copied the records
  CHK( hipMemcpy( hg.data(), dg, sizeof(gat), hipMemcpyDeviceToHost ) );
  printf( "done\n" );
  return 0;
}
