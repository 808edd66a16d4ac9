// PCIe gather probe, round 4: does the host memory type of the in region (where the GPU reads the records) or
// of the out region (where it writes them back) change what a record gather with write-back moves?  The
// stream's two tiles reach ~30 GB/s each way together (profiles/r04/final); fabric counters on
// tools/gatherprobe show 128-B read requests but 64-B write requests (profiles/r04/v).
//
// Each case: in region x out region allocation, one gather of N records (one wave per record, 4 records per
// 256-lane group, as fd_gather_kernel<4>), and the same split over two streams at once (two tiles).
//
// build: hipcc --offload-arch=gfx950 -O3 -o tools/gatherprobe/gather_memtype tools/gatherprobe/gather_memtype.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CHK(x) do { hipError_t e_ = (x); if( e_ != hipSuccess ) { fprintf( stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString( e_ ) ); exit( 1 ); } } while( 0 )

struct gat { unsigned long src; unsigned dst; unsigned sz; };

__global__ void __launch_bounds__( 256 ) gw4( gat const * g, unsigned n, unsigned char * arena, unsigned char * out ) {
  unsigned t = blockIdx.x * 4u + ( threadIdx.x >> 6 );
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
  uint4 * o = (uint4 *)( out + r.dst );
  if( l < q ) o[l] = v0;
  if( l + 64u < q ) o[l+64u] = v1;
}

enum { A_HM = 0, A_HM_COH, A_HM_NONCOH, A_REG, A_REG_COARSE, A_N };
static char const * aname[] = { "hostmalloc", "hm_coherent", "hm_noncoh", "register", "reg_coarse" };

static unsigned char * alloc_host( int kind, size_t sz, unsigned char ** dev ) {
  unsigned char * p = NULL;
  unsigned flags[] = { hipHostMallocMapped, hipHostMallocMapped | hipHostMallocCoherent,
                       hipHostMallocMapped | hipHostMallocNonCoherent };
  if( kind <= A_HM_NONCOH ) {
    CHK( hipHostMalloc( (void **)&p, sz, flags[kind] ) );
  } else {
    p = (unsigned char *)aligned_alloc( 2UL << 20, ( sz + ( 2UL << 20 ) - 1 ) & ~( ( 2UL << 20 ) - 1 ) );
    if( !p ) { fprintf( stderr, "alloc\n" ); exit( 1 ); }
    memset( p, 0, sz );
    CHK( hipHostRegister( p, sz, hipHostRegisterMapped | ( kind == A_REG_COARSE ? hipExtHostRegisterCoarseGrained : 0u ) ) );
  }
  CHK( hipHostGetDevicePointer( (void **)dev, p, 0 ) );
  return p;
}

static void free_host( int kind, unsigned char * p ) {
  if( kind <= A_HM_NONCOH ) CHK( hipHostFree( p ) );
  else { CHK( hipHostUnregister( p ) ); free( p ); }
}

int main( void ) {
  unsigned const REC = 1312, STRIDE = 1344, REPS = 20;
  unsigned long const maxn = 32768;
  unsigned sizes[] = { 4096, 16384 };
  unsigned char * arena; CHK( hipMalloc( (void **)&arena, maxn * STRIDE ) );
  gat * dg; CHK( hipMalloc( (void **)&dg, maxn * sizeof(gat) ) );
  hipStream_t st[2]; for( int i=0; i<2; i++ ) CHK( hipStreamCreateWithFlags( &st[i], hipStreamNonBlocking ) );
  hipEvent_t e0, e1; CHK( hipEventCreate( &e0 ) ); CHK( hipEventCreate( &e1 ) );
  printf( "%-12s %-12s %7s %8s %10s %10s\n", "in", "out", "streams", "records", "us/round", "GB/s(rec)" );
  int in_kinds[] = { A_HM, A_REG, A_REG_COARSE };
  for( int ik : in_kinds ) {
    unsigned char * din; unsigned char * hin = alloc_host( ik, maxn * STRIDE * 2, &din );
    memset( hin, 7, maxn * STRIDE * 2 );
    std::vector<gat> hg( maxn );
    srand( 1 );
    for( unsigned long i=0; i<maxn; i++ ) {   // records scattered over a 2x larger in region
      unsigned long c = ( i * 2 + ( rand() & 1 ) ) * STRIDE;
      hg[i].src = (unsigned long)( din + c ); hg[i].dst = (unsigned)( i * STRIDE ); hg[i].sz = REC;
    }
    CHK( hipMemcpy( dg, hg.data(), maxn * sizeof(gat), hipMemcpyHostToDevice ) );
    for( int ok = 0; ok < A_N; ok++ ) {
      unsigned char * dout; unsigned char * hout = alloc_host( ok, maxn * STRIDE, &dout );
      for( unsigned n : sizes ) {
        for( int ns = 1; ns <= 2; ns++ ) {
          auto run = [&]() {
            unsigned per = n / ns;
            for( int s=0; s<ns; s++ )
              gw4<<<( per + 3 ) / 4, 256, 0, st[s]>>>( dg + s*per, per, arena, dout );
          };
          run(); for( int s=0; s<2; s++ ) CHK( hipStreamSynchronize( st[s] ) );
          CHK( hipEventRecord( e0, st[0] ) );
          if( ns == 2 ) CHK( hipStreamWaitEvent( st[1], e0, 0 ) );
          for( unsigned r=0; r<REPS; r++ ) run();
          hipEvent_t e2; CHK( hipEventCreate( &e2 ) );
          if( ns == 2 ) { CHK( hipEventRecord( e2, st[1] ) ); CHK( hipStreamWaitEvent( st[0], e2, 0 ) ); }
          CHK( hipEventRecord( e1, st[0] ) );
          CHK( hipEventSynchronize( e1 ) );
          CHK( hipEventDestroy( e2 ) );
          float ms; CHK( hipEventElapsedTime( &ms, e0, e1 ) );
          double us = ms * 1e3 / REPS;
          printf( "%-12s %-12s %7d %8u %10.1f %10.2f\n", aname[ik], aname[ok], ns, n, us, (double)n * REC / ( us * 1e3 ) );
        }
      }
      // the records arrived in the out region (first bytes of the first record)
      if( hout[0] != 7 || hout[REC-1] != 7 ) printf( "  !! out region %s: write-back not visible (%u %u)\n", aname[ok], hout[0], hout[REC-1] );
      free_host( ok, hout );
    }
    free_host( ik, hin );
  }
  printf( "done\n" );
  return 0;
}
