// How long does a small kernel (or copy) wait to start while long verify kernels fill the GPU?
//
// The configs[4] stream's zero-copy intake copies each frag with fd_gather_kernel shortly after
// during_frag, on a high-priority stream; under full load (bench stream max leg) those copies started
// 5-18 ms after their launch even with CUs reserved for them (profiles/r03/stream_gcu).  This probe
// rebuilds the situation without the tile, one ingredient at a time: streams A and A2 keep "busy"
// kernels in flight -- 256-thread blocks that hold 204 VGPRs and spin for a fixed time, like the DSM of
// a tile's batch, at most `depth` queued per stream -- while the host issues an op on stream B every
// 100 us and records when it starts (s_memrealtime of block 0 into pinned memory, against the launch
// time on the host clock).
//
// argv[1]: flags
//   i   idle: no busy kernels (the floor)
//   h   B high priority (else normal)
//   c   CU masks: A, A2 on all CUs but the last 16, B only on those 16 (hipExtStreamCreateWithCUMask)
//   g   B's op is a gather: one 64-lane block per 1312-byte record read from pinned host memory over
//       PCIe into device memory and back into a pinned host "out dcache" (fd_gather_kernel's traffic),
//       `recs` records (argv[4]); else a one-wave probe kernel
//   e   before each busy kernel, A (A2) waits for an event recorded on B (the batch waits for its
//       gathers: hipEventRecord + hipStreamWaitEvent, as slot_launch does)
//   m   each busy kernel comes with a 1-MB H2D copy before and a 64-KB D2H copy after it on its stream
//       (the batch's descriptor upload and result download)
// argv[2]: busy blocks per kernel (512 = 2 waves per SIMD: one kernel fills the chip), argv[3]: busy
// kernel length in us, argv[4]: records per gather (g), argv[5]: busy kernels queued per stream
//
// build: hipcc --offload-arch=gfx950 -O3 -o tools/dispatchprobe/dispatch_probe tools/dispatchprobe/dispatch_probe.hip
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <ctime>
#include <vector>

#define CHK(x) do { hipError_t e_ = (x); if( e_ != hipSuccess ) { fprintf( stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString( e_ ) ); exit( 1 ); } } while( 0 )

static unsigned long now_ns() { timespec t; clock_gettime( CLOCK_MONOTONIC, &t ); return (unsigned long)t.tv_sec * 1000000000UL + t.tv_nsec; }

// busy: spin for `ticks` of the 100-MHz clock while keeping ~200 VGPRs live (a DSM-like footprint)
__global__ void __launch_bounds__( 256 ) busy( unsigned long ticks, unsigned * sink ) {
  unsigned v[ 100 ];
#pragma unroll
  for( int i=0; i<100; i++ ) v[i] = threadIdx.x * 7u + (unsigned)i;
  unsigned long t0 = __builtin_amdgcn_s_memrealtime();
  while( __builtin_amdgcn_s_memrealtime() - t0 < ticks ) {
#pragma unroll
    for( int i=0; i<100; i++ ) v[i] = v[i] * 0x9e3779b1u + v[( i + 1 ) % 100];
  }
  unsigned x = 0u;
#pragma unroll
  for( int i=0; i<100; i++ ) x ^= v[i];
  if( x == 0x12345678u ) sink[ threadIdx.x ] = x;
}

__global__ void __launch_bounds__( 64 ) probe( unsigned long * out ) {
  if( threadIdx.x == 0 ) __hip_atomic_store( out, __builtin_amdgcn_s_memrealtime(), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM );
}

// fd_gather_kernel's traffic: record b (82 x 16 B) from host src into device arena and host out
__global__ void __launch_bounds__( 64 ) gather( uint4 const * src, uint4 * arena, uint4 * out, unsigned long * t ) {
  if( blockIdx.x == 0 && threadIdx.x == 0 ) __hip_atomic_store( t, __builtin_amdgcn_s_memrealtime(), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM );
  unsigned b = blockIdx.x, i = threadIdx.x;
  uint4 const * s = src + (size_t)b * 88;
  uint4 v0 = s[i], v1 = make_uint4( 0, 0, 0, 0 );
  if( i < 18 ) v1 = s[i + 64];
  arena[ (size_t)b * 88 + i ] = v0; out[ (size_t)b * 88 + i ] = v0;
  if( i < 18 ) { arena[ (size_t)b * 88 + i + 64 ] = v1; out[ (size_t)b * 88 + i + 64 ] = v1; }
}

int main( int argc, char ** argv ) {
  char const * fl = argc > 1 ? argv[1] : "h";
  int blocks = argc > 2 ? atoi( argv[2] ) : 512;
  unsigned long busy_us = argc > 3 ? strtoul( argv[3], 0, 10 ) : 4000UL;
  int recs = argc > 4 ? atoi( argv[4] ) : 1024;
  int depth = argc > 5 ? atoi( argv[5] ) : 2;
  bool idle = strchr( fl, 'i' ), hi = strchr( fl, 'h' ), cum = strchr( fl, 'c' ), gat = strchr( fl, 'g' );
  bool ev = strchr( fl, 'e' ), mc = strchr( fl, 'm' );
  CHK( hipSetDevice( 0 ) );
  int ncu = 0; CHK( hipDeviceGetAttribute( &ncu, hipDeviceAttributeMultiprocessorCount, 0 ) );
  int lo = 0, hip_hi = 0; CHK( hipDeviceGetStreamPriorityRange( &lo, &hip_hi ) );
  hipStream_t A[2], B;
  if( cum ) {
    std::vector<uint32_t> am( ( ncu + 31 ) / 32, 0u ), bm( am.size(), 0u );
    for( int c=0; c<ncu; c++ ) ( c >= ncu - 16 ? bm : am )[ c / 32 ] |= 1u << ( c % 32 );
    for( int k=0; k<2; k++ ) CHK( hipExtStreamCreateWithCUMask( &A[k], (uint32_t)am.size(), am.data() ) );
    CHK( hipExtStreamCreateWithCUMask( &B, (uint32_t)bm.size(), bm.data() ) );
  } else {
    for( int k=0; k<2; k++ ) CHK( hipStreamCreateWithFlags( &A[k], hipStreamNonBlocking ) );
    CHK( hipStreamCreateWithPriority( &B, hipStreamNonBlocking, hi ? hip_hi : lo ) );
  }
  enum { NP = 2000, RING = 16 };
  unsigned long * h; CHK( hipHostMalloc( (void **)&h, ( NP + 1 ) * sizeof(unsigned long), hipHostMallocDefault ) );
  unsigned long * d; CHK( hipHostGetDevicePointer( (void **)&d, h, 0 ) );
  unsigned * sink; CHK( hipMalloc( &sink, 4096 ) );
  size_t gbytes = (size_t)recs * 88 * 16;
  unsigned char * hsrc, * hout, * dsrc, * dout, * arena;
  CHK( hipHostMalloc( (void **)&hsrc, gbytes, hipHostMallocDefault ) );
  CHK( hipHostMalloc( (void **)&hout, gbytes, hipHostMallocDefault ) );
  CHK( hipHostGetDevicePointer( (void **)&dsrc, hsrc, 0 ) );
  CHK( hipHostGetDevicePointer( (void **)&dout, hout, 0 ) );
  CHK( hipMalloc( &arena, gbytes ) );
  unsigned char * hm, * dm; CHK( hipHostMalloc( (void **)&hm, 1 << 20, hipHostMallocDefault ) ); CHK( hipMalloc( &dm, 1 << 20 ) );
  memset( hsrc, 1, gbytes );
  hipEvent_t evb; CHK( hipEventCreateWithFlags( &evb, hipEventDisableTiming ) );
  hipEvent_t done[2][ RING ];
  for( int k=0; k<2; k++ ) for( int j=0; j<RING; j++ ) CHK( hipEventCreateWithFlags( &done[k][j], hipEventDisableTiming ) );
  // clock calibration: GPU 100-MHz ticks vs host ns (idle device, best of 5 round trips)
  double off = 0., best = 1e30;
  for( int k=0; k<5; k++ ) {
    h[NP] = 0;
    unsigned long t0 = now_ns();
    hipLaunchKernelGGL( probe, dim3(1), dim3(64), 0, B, d + NP );
    CHK( hipStreamSynchronize( B ) );
    unsigned long t1 = now_ns();
    if( (double)( t1 - t0 ) < best ) { best = (double)( t1 - t0 ); off = (double)h[NP] * 10.0 - 0.5 * ( (double)t0 + (double)t1 ); }
  }
  hipLaunchKernelGGL( busy, dim3(blocks), dim3(256), 0, A[0], 1000UL, sink );
  hipLaunchKernelGGL( gather, dim3(recs), dim3(64), 0, B, (uint4 const *)dsrc, (uint4 *)arena, (uint4 *)dout, d + NP );
  CHK( hipDeviceSynchronize() );
  unsigned long nb[2] = { 0, 0 }, nd[2] = { 0, 0 }, nbusy = 0;
  std::vector<unsigned long> tl( NP );
  unsigned long t_begin = now_ns();
  for( int i=0; i<NP; i++ ) {
    unsigned long t = now_ns();
    for( int k=0; k<2 && !idle; k++ ) {                 // keep `depth` busy kernels queued per stream
      while( nd[k] < nb[k] && hipEventQuery( done[k][ nd[k] % RING ] ) == hipSuccess ) nd[k]++;
      while( nb[k] - nd[k] < (unsigned long)depth ) {
        if( ev ) { CHK( hipEventRecord( evb, B ) ); CHK( hipStreamWaitEvent( A[k], evb, 0 ) ); }
        if( mc ) CHK( hipMemcpyAsync( dm, hm, 1 << 20, hipMemcpyHostToDevice, A[k] ) );
        hipLaunchKernelGGL( busy, dim3(blocks), dim3(256), 0, A[k], busy_us * 100UL, sink );
        if( mc ) CHK( hipMemcpyAsync( hm, dm, 1 << 16, hipMemcpyDeviceToHost, A[k] ) );
        CHK( hipEventRecord( done[k][ nb[k] % RING ], A[k] ) );
        nb[k]++; nbusy++;
      }
    }
    h[i] = 0;
    tl[i] = now_ns();
    if( gat ) hipLaunchKernelGGL( gather, dim3(recs), dim3(64), 0, B, (uint4 const *)dsrc, (uint4 *)arena, (uint4 *)dout, d + i );
    else      hipLaunchKernelGGL( probe, dim3(1), dim3(64), 0, B, d + i );
    while( now_ns() - t < 100000UL ) {}
  }
  double wall = ( now_ns() - t_begin ) * 1e-9;
  CHK( hipDeviceSynchronize() );
  std::vector<double> dl;
  for( int i=0; i<NP; i++ ) if( h[i] ) dl.push_back( ( (double)h[i] * 10.0 - off - (double)tl[i] ) * 1e-3 );
  std::sort( dl.begin(), dl.end() );
  auto q = [&]( double p ) { return dl.empty() ? -1. : dl[ std::min( dl.size() - 1, (size_t)( p * dl.size() ) ) ]; };
  printf( "{\"flags\": \"%s\", \"busy_blocks\": %d, \"busy_us\": %lu, \"recs\": %d, \"depth\": %d, \"busy_kernels\": %lu, "
          "\"n\": %zu, \"delay_us\": {\"p50\": %.1f, \"p90\": %.1f, \"p99\": %.1f, \"max\": %.1f}, \"busy_per_s\": %.0f}\n",
          fl, blocks, busy_us, recs, depth, nbusy, dl.size(), q( .5 ), q( .9 ), q( .99 ), dl.empty() ? -1. : dl.back(),
          nbusy / wall );
  return 0;
}
