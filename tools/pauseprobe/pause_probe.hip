// Do GPU-side pauses show without this repository's engine, tile or PyTorch?  The paced stream legs of
// bench.py meet pauses of ~1 ms that hold every queue, on a 100 ms grid, on some boxes.
// This probe is plain HIP: it launches a one-wave kernel on one stream every `period` us for `seconds`
// and records when each starts (s_memrealtime of its lane 0, stored with a vector store into pinned host
// memory) against its launch on the host clock.  Mode 'b': two other streams keep 300-us kernels of 256
// blocks in flight (half the CUs busy, like a paced tile's walks); mode 'i': the GPU otherwise idle.
// Output: one JSON line -- delay quantiles and the episodes of delays over 250 us (start ms from the
// first launch, longest delay us, launches), so a 100-ms grid shows in the start times.
//
// build: hipcc --offload-arch=gfx950 -O3 -o tools/pauseprobe/pause_probe tools/pauseprobe/pause_probe.hip
// usage: tools/pauseprobe/pause_probe <i|b> [seconds=5] [period_us=50]
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <ctime>
#include <vector>

#define CHK(x) do { hipError_t e_ = (x); if( e_ != hipSuccess ) { fprintf( stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString( e_ ) ); exit( 1 ); } } while( 0 )

static unsigned long now_ns( void ) {
  timespec ts; clock_gettime( CLOCK_MONOTONIC, &ts ); return (unsigned long)ts.tv_sec * 1000000000UL + (unsigned long)ts.tv_nsec;
}

__global__ void probe( unsigned long * out ) {
  if( threadIdx.x == 0 ) out[0] = __builtin_amdgcn_s_memrealtime();
}

__global__ void busy( unsigned long ticks, unsigned * sink ) {   // spins `ticks` of the 100-MHz clock
  unsigned long t0 = __builtin_amdgcn_s_memrealtime();
  unsigned x = threadIdx.x;
  while( __builtin_amdgcn_s_memrealtime() - t0 < ticks ) x = x * 1664525u + 1013904223u;
  if( x == 0x12345678u ) sink[ threadIdx.x ] = x;
}

int main( int argc, char ** argv ) {
  bool load = argc > 1 && argv[1][0] == 'b';
  double seconds = argc > 2 ? atof( argv[2] ) : 5.0;
  unsigned long period = argc > 3 ? strtoul( argv[3], 0, 10 ) : 50UL;
  size_t NP = (size_t)( seconds * 1e6 / (double)period );
  if( NP < 16 || NP > 2000000 ) { fprintf( stderr, "bad seconds / period\n" ); return 2; }
  CHK( hipSetDevice( 0 ) );
  hipStream_t B, A[2];
  CHK( hipStreamCreateWithFlags( &B, hipStreamNonBlocking ) );
  for( int k=0; k<2; k++ ) CHK( hipStreamCreateWithFlags( &A[k], hipStreamNonBlocking ) );
  unsigned long * h; CHK( hipHostMalloc( (void **)&h, ( NP + 1 ) * sizeof(unsigned long), hipHostMallocDefault ) );
  memset( h, 0, ( NP + 1 ) * sizeof(unsigned long) );
  unsigned long * d; CHK( hipHostGetDevicePointer( (void **)&d, h, 0 ) );
  unsigned * sink; CHK( hipMalloc( &sink, 4096 ) );
  enum { RING = 8 };
  hipEvent_t done[2][ RING ];
  for( int k=0; k<2; k++ ) for( int j=0; j<RING; j++ ) CHK( hipEventCreateWithFlags( &done[k][j], hipEventDisableTiming ) );
  double off = 0., best = 1e30;                     // GPU clock (10 ns ticks) vs host ns: best of 9 round trips
  for( int k=0; k<9; k++ ) {
    h[NP] = 0;
    unsigned long t0 = now_ns();
    hipLaunchKernelGGL( probe, dim3(1), dim3(64), 0, B, d + NP );
    CHK( hipStreamSynchronize( B ) );
    unsigned long t1 = now_ns();
    if( (double)( t1 - t0 ) < best ) { best = (double)( t1 - t0 ); off = (double)h[NP] * 10.0 - 0.5 * ( (double)t0 + (double)t1 ); }
  }
  std::vector<unsigned long> tl( NP );
  unsigned long nb[2] = { 0, 0 }, nd[2] = { 0, 0 };
  unsigned long t_begin = now_ns();
  for( size_t i=0; i<NP; i++ ) {
    unsigned long t = t_begin + (unsigned long)i * period * 1000UL;
    while( now_ns() < t ) {}
    for( int k=0; k<2 && load; k++ ) {              // two 300-us kernels of 256 blocks in flight per stream
      while( nd[k] < nb[k] && hipEventQuery( done[k][ nd[k] % RING ] ) == hipSuccess ) nd[k]++;
      while( nb[k] - nd[k] < 2UL ) {
        hipLaunchKernelGGL( busy, dim3(256), dim3(256), 0, A[k], 30000UL, sink );
        CHK( hipEventRecord( done[k][ nb[k] % RING ], A[k] ) );
        nb[k]++;
      }
    }
    tl[i] = now_ns();
    hipLaunchKernelGGL( probe, dim3(1), dim3(64), 0, B, d + i );
  }
  CHK( hipDeviceSynchronize() );
  std::vector<double> dl( NP, -1. );
  std::vector<double> s;
  for( size_t i=0; i<NP; i++ ) if( h[i] ) { dl[i] = ( (double)h[i] * 10.0 - off - (double)tl[i] ) * 1e-3; s.push_back( dl[i] ); }
  std::sort( s.begin(), s.end() );
  auto q = [&]( double p ) { return s.empty() ? -1. : s[ std::min( s.size() - 1, (size_t)( p * s.size() ) ) ]; };
  printf( "{\"mode\": \"%s\", \"seconds\": %.2f, \"period_us\": %lu, \"n\": %zu, \"delay_us\": {\"p50\": %.1f, \"p99\": %.1f, "
          "\"p999\": %.1f, \"max\": %.1f}, \"episodes\": [", load ? "busy" : "idle", seconds, period, s.size(), q( .5 ), q( .99 ),
          q( .999 ), s.empty() ? -1. : s.back() );
  int ne = 0; double e_start = 0., e_max = 0.; unsigned long e_n = 0, e_last = 0;   // episodes: hits < 5 ms apart
  for( size_t i=0; i<NP; i++ ) {
    if( !( dl[i] > 250. ) ) continue;
    unsigned long ti = tl[i] - tl[0];
    if( e_n && ti - e_last > 5000000UL ) {
      if( ne < 200 ) printf( "%s[%.2f, %.0f, %lu]", ne ? ", " : "", e_start * 1e-6, e_max, e_n );
      ne++; e_n = 0; e_max = 0.;
    }
    if( !e_n ) e_start = (double)ti;
    e_n++; e_last = ti; if( dl[i] > e_max ) e_max = dl[i];
  }
  if( e_n ) { if( ne < 200 ) printf( "%s[%.2f, %.0f, %lu]", ne ? ", " : "", e_start * 1e-6, e_max, e_n ); ne++; }
  printf( "], \"n_episodes\": %d}\n", ne );
  return 0;
}
