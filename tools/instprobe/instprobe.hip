// Issue-rate probe for single VALU instructions on gfx950: every lane runs
// 16 independent chains of one instruction (inline asm, so the compiler
// cannot rewrite it), 8 waves per SIMD over the whole chip.  Prints, per
// instruction kind, G lane-ops / s, the shader clock the kernel ran at
// (s_memtime cycles over s_memrealtime's 100 MHz ticks, sampled by one
// lane per block at its start and end) and the resulting cycles per
// wave64 instruction per SIMD -- the figure MI355X_MICROARCH.md's cycle
// table gives as 2 for v_fma_f32 (SIMD-32).
// build: hipcc --offload-arch=gfx950 -O3 -o tools/instprobe/instprobe tools/instprobe/instprobe.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

#define CH 16
/* clk[4*block..]: memtime start, memtime end, realtime start, realtime end */
#define CLK_START unsigned long long c0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
#define CLK_END   if( threadIdx.x == 0 ) { unsigned long long c1 = __builtin_amdgcn_s_memtime(),              \
                    r1 = __builtin_amdgcn_s_memrealtime(); unsigned long long * o = clk + 4 * blockIdx.x;      \
                    o[0] = c0; o[1] = c1; o[2] = r0; o[3] = r1; }
#define DEF_K( NAME, BODY )                                                         \
__global__ void __launch_bounds__( 256 ) NAME( unsigned iters, unsigned seed, unsigned * out, unsigned long long * clk ) { \
  CLK_START                                                                         \
  unsigned v[CH];                                                                   \
  _Pragma("unroll") for( int c=0; c<CH; c++ ) v[c] = seed + threadIdx.x * 7u + c;    \
  for( unsigned i=0; i<iters; i++ ) {                                               \
    _Pragma("unroll") for( int c=0; c<CH; c++ ) { BODY; }                           \
  }                                                                                 \
  unsigned r = 0; _Pragma("unroll") for( int c=0; c<CH; c++ ) r ^= v[c];             \
  if( r == 0x12345678u ) out[0] = r;                                                \
  CLK_END                                                                           \
}
DEF_K( k_add,    asm volatile( "v_add_u32 %0, %0, %1" : "+v"( v[c] ) : "v"( seed ) ) )
DEF_K( k_addself,asm volatile( "v_add_u32 %0, %0, %0" : "+v"( v[c] ) ) )
DEF_K( k_lshl,   asm volatile( "v_lshlrev_b32 %0, 1, %0" : "+v"( v[c] ) ) )
DEF_K( k_and,    asm volatile( "v_and_b32 %0, %0, %1" : "+v"( v[c] ) : "v"( seed ) ) )
DEF_K( k_mullo,  asm volatile( "v_mul_lo_u32 %0, %0, 19" : "+v"( v[c] ) ) )
DEF_K( k_mad24,  asm volatile( "v_mad_u32_u24 %0, %0, 19, %1" : "+v"( v[c] ) : "v"( seed ) ) )
DEF_K( k_align,  asm volatile( "v_alignbit_b32 %0, %0, %1, 7" : "+v"( v[c] ) : "v"( seed ) ) )
DEF_K( k_bitop3, asm volatile( "v_bitop3_b32 %0, %0, %1, %1 bitop3:0x96" : "+v"( v[c] ) : "v"( seed ) ) )
DEF_K( k_cndmask,asm volatile( "v_cmp_gt_u32 vcc, 3, %1\n\tv_cndmask_b32 %0, %0, %1, vcc" : "+v"( v[c] ) : "v"( threadIdx.x ) : "vcc" ) )
DEF_K( k_cndsel, unsigned m = threadIdx.x & 1u; v[c] = m ? v[c] + seed : v[c] ^ seed )
DEF_K( k_dpp,    asm volatile( "v_mov_b32_dpp %0, %0 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf" : "+v"( v[c] ) ) )
DEF_K( k_lshladd,asm volatile( "v_lshl_add_u32 %0, %0, 4, %1" : "+v"( v[c] ) : "v"( seed ) ) )
DEF_K( k_fma,    asm volatile( "v_fma_f32 %0, %0, %1, %1" : "+v"( v[c] ) : "v"( seed ) ) )
DEF_K( k_addf,   asm volatile( "v_add_f32 %0, %0, %1" : "+v"( v[c] ) : "v"( seed ) ) )
DEF_K( k_mul24,  asm volatile( "v_mul_u32_u24 %0, %0, %1" : "+v"( v[c] ) : "v"( seed ) ) )
DEF_K( k_sub,    asm volatile( "v_sub_u32 %0, %1, %0" : "+v"( v[c] ) : "v"( seed ) ) )
DEF_K( k_mov,    asm volatile( "v_mov_b32 %0, %1" : "=v"( v[c] ) : "v"( v[(c+1)%CH] ) ) )
DEF_K( k_lshr,   asm volatile( "v_lshrrev_b32 %0, 3, %0" : "+v"( v[c] ) ) )
DEF_K( k_snop,   asm volatile( "s_nop 0" ::: ); v[c] ^= seed )

__global__ void __launch_bounds__( 256 ) k_mad64( unsigned iters, unsigned seed, unsigned * out, unsigned long long * clk ) {
  CLK_START
  uint64_t v[CH / 2];
  for( int c=0; c<CH/2; c++ ) v[c] = seed + threadIdx.x * 7u + c;
  for( unsigned i=0; i<iters; i++ ) {
#pragma unroll
    for( int c=0; c<CH/2; c++ ) asm volatile( "v_mad_u64_u32 %0, vcc, %1, %1, %0" : "+v"( v[c] ) : "v"( seed ) : "vcc" );
  }
  uint64_t r = 0; for( int c=0; c<CH/2; c++ ) r ^= v[c];
  if( r == 0x12345678u ) out[0] = (unsigned)r;
  CLK_END
}
__global__ void __launch_bounds__( 256 ) k_lshladd64( unsigned iters, unsigned seed, unsigned * out, unsigned long long * clk ) {
  CLK_START
  uint64_t v[CH / 2];
  for( int c=0; c<CH/2; c++ ) v[c] = seed + threadIdx.x * 7u + c;
  uint64_t sv = seed;
  for( unsigned i=0; i<iters; i++ ) {
#pragma unroll
    for( int c=0; c<CH/2; c++ ) asm volatile( "v_lshl_add_u64 %0, %0, 1, %1" : "+v"( v[c] ) : "v"( sv ) );
  }
  uint64_t r = 0; for( int c=0; c<CH/2; c++ ) r ^= v[c];
  if( r == 0x12345678u ) out[0] = (unsigned)r;
  CLK_END
}
__global__ void __launch_bounds__( 256 ) k_fma64( unsigned iters, unsigned seed, unsigned * out, unsigned long long * clk ) {
  CLK_START
  double v[CH / 2];
  for( int c=0; c<CH/2; c++ ) v[c] = (double)( seed + threadIdx.x * 7u + c );
  double sv = (double)seed * 1e-9;
  for( unsigned i=0; i<iters; i++ ) {
#pragma unroll
    for( int c=0; c<CH/2; c++ ) asm volatile( "v_fma_f64 %0, %0, %1, %1" : "+v"( v[c] ) : "v"( sv ) );
  }
  double r = 0; for( int c=0; c<CH/2; c++ ) r += v[c];
  if( r == 0.125 ) out[0] = 1u;
  CLK_END
}
__global__ void __launch_bounds__( 256 ) k_lshr64( unsigned iters, unsigned seed, unsigned * out, unsigned long long * clk ) {
  CLK_START
  uint64_t v[CH / 2];
  for( int c=0; c<CH/2; c++ ) v[c] = seed + threadIdx.x * 7u + c;
  for( unsigned i=0; i<iters; i++ ) {
#pragma unroll
    for( int c=0; c<CH/2; c++ ) asm volatile( "v_lshrrev_b64 %0, 1, %0" : "+v"( v[c] ) );
  }
  uint64_t r = 0; for( int c=0; c<CH/2; c++ ) r ^= v[c];
  if( r == 0x12345678u ) out[0] = (unsigned)r;
  CLK_END
}

typedef void (*kfn)( unsigned, unsigned, unsigned *, unsigned long long * );
int main() {
  struct { char const * name; kfn f; int per; } ks[] = {
    { "v_add_u32",         k_add,     CH }, { "v_add_u32 (x+x)", k_addself, CH }, { "v_lshlrev_b32", k_lshl, CH },
    { "v_and_b32",         k_and,     CH }, { "v_mul_lo_u32",    k_mullo,   CH }, { "v_mad_u32_u24", k_mad24, CH },
    { "v_alignbit_b32",    k_align,   CH }, { "v_bitop3_b32",    k_bitop3,  CH }, { "v_cmp+v_cndmask", k_cndmask, CH },
    { "sel (compiler)", k_cndsel, CH }, { "v_mov_b32_dpp", k_dpp, CH }, { "v_lshl_add_u32", k_lshladd, CH },
    { "v_mad_u64_u32",     k_mad64, CH/2 }, { "v_lshrrev_b64",   k_lshr64, CH/2 },
    { "v_fma_f32",         k_fma,   CH }, { "v_add_f32",       k_addf,    CH }, { "v_mul_u32_u24", k_mul24, CH },
    { "v_sub_u32",         k_sub,   CH }, { "v_mov_b32",       k_mov,     CH }, { "v_lshrrev_b32", k_lshr, CH },
    { "s_nop 0 (+v_xor)",  k_snop,  CH }, { "v_lshl_add_u64",  k_lshladd64, CH/2 }, { "v_fma_f64", k_fma64, CH/2 } };
  int ncu = 0; hipDeviceGetAttribute( &ncu, hipDeviceAttributeMultiprocessorCount, 0 );
  unsigned * out; hipMalloc( &out, 4 );
  unsigned iters = 4096; int blocks = ncu * 8;        /* 8 x 256 threads per CU = 8 waves per SIMD */
  unsigned long long * clk; hipMalloc( &clk, (size_t)blocks * 4 * sizeof(unsigned long long) );
  unsigned long long * hc = (unsigned long long *)malloc( (size_t)blocks * 4 * sizeof(unsigned long long) );
  hipEvent_t a, b; hipEventCreate( &a ); hipEventCreate( &b );
  printf( "%-18s %12s %10s %12s %14s\n", "instruction", "G lane-op/s", "clock MHz", "cyc/wave-op", "G lane-op/s@2.4" );
  for( auto & k : ks ) {
    hipLaunchKernelGGL( k.f, dim3(blocks), dim3(256), 0, 0, 16u, 1u, out, clk );
    float best = 1e30f; double mhz = 0.;
    for( int r=0; r<3; r++ ) {
      hipEventRecord( a ); hipLaunchKernelGGL( k.f, dim3(blocks), dim3(256), 0, 0, iters, 1u, out, clk ); hipEventRecord( b );
      hipEventSynchronize( b ); float ms; hipEventElapsedTime( &ms, a, b );
      if( ms < best ) {
        best = ms;
        hipMemcpy( hc, clk, (size_t)blocks * 4 * sizeof(unsigned long long), hipMemcpyDeviceToHost );
        double dc = 0., dr = 0.;
        for( int i=0; i<blocks; i++ ) { dc += (double)( hc[4*i+1] - hc[4*i] ); dr += (double)( hc[4*i+3] - hc[4*i+2] ); }
        mhz = dr > 0. ? dc / dr * 100. : 0.;        /* s_memrealtime: 100 MHz */
      }
    }
    double ops = (double)blocks * 256.0 * iters * k.per;
    double rate = ops / ( best * 1e-3 );
    /* per SIMD: (blocks*4 waves / (ncu*4 SIMDs)) waves each issuing iters*per wave-instructions */
    double wave_ops_per_simd = (double)blocks * 4.0 / ( (double)ncu * 4.0 ) * iters * k.per;
    double cyc = mhz * 1e6 * best * 1e-3 / wave_ops_per_simd;
    printf( "%-18s %12.1f %10.0f %12.2f %14.1f\n", k.name, rate * 1e-9, mhz, cyc, ( (double)ncu * 4.0 * 64.0 * 2.4e9 / cyc ) * 1e-9 );
  }
  return 0;
}
