/* fieldbench.hip -- microbenchmark of GF(2^255-19) multiply/square
   formulations on gfx950 (design exploration tool, not product code).

   Each lane runs two independent dependent chains (x = x*y, u = u*v) of
   ITERS operations, full grid; prints Gop/s for each variant and checks
   all variants agree (mod p) on the final values. */
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#include <string.h>

#define FD_GPU_MUL_ASM 1
#include "../../firedancer_amd/csrc/fd_gpu_f25519.h"

/* ---- variant B: 8x32 operand scanning in plain C ---------------------- */
FD_DEV void mulB( fe & r, fe const & a, fe const & b ) {
  u32 t[16];
  { u64 c = 0;
#pragma unroll
    for( int j=0; j<8; j++ ) { c = fd_mad( a.v[0], b.v[j], c ); t[j] = (u32)c; c >>= 32; }
    t[8] = (u32)c; }
#pragma unroll
  for( int i=1; i<8; i++ ) {
    u64 c = 0;
#pragma unroll
    for( int j=0; j<8; j++ ) { c = fd_mad( a.v[i], b.v[j], (u64)t[i+j] + c ); t[i+j] = (u32)c; c >>= 32; }
    t[i+8] = (u32)c;
  }
  fe_fold512( r, t );
}

/* ---- variant C: radix 2^25.5 (10 limbs 26/25 bits in u32 registers) ---- */
struct f10 { u32 v[10]; };

FD_DEV void carry10( f10 & r, u64 h[10] ) {
  /* limb i holds 26 bits if i even else 25 */
  u64 c;
#pragma unroll
  for( int pass=0; pass<1; pass++ ) {
    c = h[0] >> 26; h[1] += c; h[0] &= 0x3ffffffUL;
    c = h[4] >> 26; h[5] += c; h[4] &= 0x3ffffffUL;
    c = h[1] >> 25; h[2] += c; h[1] &= 0x1ffffffUL;
    c = h[5] >> 25; h[6] += c; h[5] &= 0x1ffffffUL;
    c = h[2] >> 26; h[3] += c; h[2] &= 0x3ffffffUL;
    c = h[6] >> 26; h[7] += c; h[6] &= 0x3ffffffUL;
    c = h[3] >> 25; h[4] += c; h[3] &= 0x1ffffffUL;
    c = h[7] >> 25; h[8] += c; h[7] &= 0x1ffffffUL;
    c = h[4] >> 26; h[5] += c; h[4] &= 0x3ffffffUL;
    c = h[8] >> 26; h[9] += c; h[8] &= 0x3ffffffUL;
    c = h[9] >> 25; h[0] += c * 19; h[9] &= 0x1ffffffUL;
    c = h[0] >> 26; h[1] += c; h[0] &= 0x3ffffffUL;
  }
#pragma unroll
  for( int i=0; i<10; i++ ) r.v[i] = (u32)h[i];
}

FD_DEV void mulC( f10 & r, f10 const & f, f10 const & g ) {
  u32 g19[10], f2[10];
#pragma unroll
  for( int i=0; i<10; i++ ) { g19[i] = 19u * g.v[i]; f2[i] = (i & 1) ? 2u * f.v[i] : f.v[i]; }
  u64 h[10];
#pragma unroll
  for( int k=0; k<10; k++ ) {
    u64 acc = 0;
#pragma unroll
    for( int i=0; i<10; i++ ) {
      int j = k - i;
      u32 fi = ((i & 1) && (j & 1 || j < 0) ) ? f2[i] : f.v[i];
      /* ref10 rule: odd i with odd j (in the wrapped index) doubles */
      int jj = j < 0 ? j + 10 : j;
      fi = ((i & 1) && (jj & 1)) ? f2[i] : f.v[i];
      u32 gj = j < 0 ? g19[jj] : g.v[jj];
      acc = fd_mad( fi, gj, acc );
    }
    h[k] = acc;
  }
  carry10( r, h );
}

FD_DEV void sqrC( f10 & r, f10 const & f ) { mulC( r, f, f ); }

/* conversions for checking */
FD_DEV void to10( f10 & r, fe const & a ) {
  fe c; fe_canon( c, a );
  u32 w[9]; for( int i=0; i<8; i++ ) w[i] = c.v[i]; w[8] = 0;
  int bit = 0;
  for( int i=0; i<10; i++ ) {
    int nb = (i & 1) ? 25 : 26;
    int wi = bit >> 5, sh = bit & 31;
    u64 x = (u64)w[wi] | ((u64)w[wi+1] << 32);
    r.v[i] = (u32)((x >> sh) & ((1UL << nb) - 1));
    bit += nb;
  }
}
FD_DEV void from10( fe & r, f10 const & a ) {
  /* value = sum a_i 2^{ceil(25.5 i)}; limbs may exceed their width slightly */
  u64 acc[9] = {0};
  fe res = fe_zero();
  int bit = 0;
  for( int i=0; i<10; i++ ) {
    int nb = (i & 1) ? 25 : 26;
    fe t = fe_zero();
    int wi = bit >> 5, sh = bit & 31;
    u64 x = (u64)a.v[i] << sh;
    t.v[wi] = (u32)x; if( wi+1 < 8 ) t.v[wi+1] = (u32)(x >> 32);
    fe_add( res, res, t );
    bit += nb;
  }
  (void)acc;
  r = res;
}

#define ITERS 2000

template<int V>
__global__ void __launch_bounds__( 256 ) kbench( u32 * out, u32 seed ) {
  fe x, y, u, v;
  for( int i=0; i<8; i++ ) {
    x.v[i] = seed * (i+1) + threadIdx.x; y.v[i] = (seed ^ 0x9e3779b9u) * (i+3) + blockIdx.x;
    u.v[i] = x.v[i] ^ 0x55555555u; v.v[i] = y.v[i] + 12345u;
  }
  x.v[7] &= 0x7fffffff; y.v[7] &= 0x7fffffff; u.v[7] &= 0x7fffffff; v.v[7] &= 0x7fffffff;
  if( V == 0 || V == 1 ) {
    for( int it=0; it<ITERS; it++ ) {
      if( V == 0 ) { fe_mul( x, x, y ); fe_mul( u, u, v ); }
      else         { mulB( x, x, y );   mulB( u, u, v ); }
    }
  } else if( V == 2 ) {
    f10 X, Y, U, W; to10( X, x ); to10( Y, y ); to10( U, u ); to10( W, v );
    for( int it=0; it<ITERS; it++ ) { mulC( X, X, Y ); mulC( U, U, W ); }
    from10( x, X ); from10( u, U );
  } else if( V == 3 ) {
    for( int it=0; it<ITERS; it++ ) { fe_sqr( x, x ); fe_sqr( u, u ); }
  } else if( V == 4 ) {
    f10 X, U; to10( X, x ); to10( U, u );
    for( int it=0; it<ITERS; it++ ) { sqrC( X, X ); sqrC( U, U ); }
    from10( x, X ); from10( u, U );
  }
  fe_canon( x, x ); fe_canon( u, u );
  size_t g = (size_t)blockIdx.x * 256 + threadIdx.x;
  for( int i=0; i<8; i++ ) { out[(g*16) + i] = x.v[i]; out[g*16 + 8 + i] = u.v[i]; }
}

template<int V>
static double run( u32 * d, int grid, u32 * h, size_t n ) {
  hipEvent_t e0, e1; hipEventCreate( &e0 ); hipEventCreate( &e1 );
  hipLaunchKernelGGL( kbench<V>, dim3(grid), dim3(256), 0, 0, d, 7u );
  hipEventRecord( e0 );
  hipLaunchKernelGGL( kbench<V>, dim3(grid), dim3(256), 0, 0, d, 7u );
  hipEventRecord( e1 ); hipEventSynchronize( e1 );
  float ms; hipEventElapsedTime( &ms, e0, e1 );
  hipMemcpy( h, d, n * 4, hipMemcpyDeviceToHost );
  double ops = (double)grid * 256 * 2 * ITERS;
  return ops / (ms * 1e-3) / 1e9;
}

int main() {
  hipDeviceProp_t p; hipGetDeviceProperties( &p, 0 );
  int grid = p.multiProcessorCount * 8;
  size_t n = (size_t)grid * 256 * 16;
  u32 * d; hipMalloc( &d, n * 4 );
  u32 * h0 = (u32*)malloc( n*4 ), * h1 = (u32*)malloc( n*4 ), * h2 = (u32*)malloc( n*4 );
  double g0 = run<0>( d, grid, h0, n );
  double g1 = run<1>( d, grid, h1, n );
  double g2 = run<2>( d, grid, h2, n );
  printf( "mul  A comba-asm   %8.1f Gmul/s\n", g0 );
  printf( "mul  B opscan-C    %8.1f Gmul/s  agree=%d\n", g1, !memcmp( h0, h1, n*4 ) );
  printf( "mul  C radix25.5   %8.1f Gmul/s  agree=%d\n", g2, !memcmp( h0, h2, n*4 ) );
  double s0 = run<3>( d, grid, h0, n );
  double s1 = run<4>( d, grid, h1, n );
  printf( "sqr  A comba-asm   %8.1f Gsqr/s\n", s0 );
  printf( "sqr  C radix25.5   %8.1f Gsqr/s  agree=%d\n", s1, !memcmp( h0, h1, n*4 ) );
  return 0;
}
