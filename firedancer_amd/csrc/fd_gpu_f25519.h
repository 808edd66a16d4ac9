#pragma once
/* fd_gpu_f25519.h -- GF(2^255-19) for CDNA4 (gfx950), one field element
   per lane, device code only.

   MI355X-native replacement for the reference's field layer
   (src/ballet/ed25519/fd_f25519.h API; AVX-512 r43x6 backend
   avx512/fd_r43x6.h, portable fiat 5x51 backend ref/fd_f25519.h).  Not a
   port of either: the reference packs ONE element into 6 lanes of a zmm
   (latency-optimised, one signature at a time); here each of the 64
   lanes of a wave owns a whole element of its own signature.

   Representation: 10 unsigned 32-bit limbs, radix 2^25.5 (limb i sits
   at bit ceil(25.5 i), 26 bits wide for even i, 25 for odd i).  Products
   are v_mad_u64_u32 (32x32+64 -> 64) accumulated carry-free in 64-bit
   column sums; one carry chain per multiply.  Measured on MI355X
   (tools/fieldbench) this beats a saturated 8x32-bit Comba multiply:
   the 10 column sums are independent chains (ILP instead of one serial
   carry chain), additions need no carry propagation at all, and a
   squaring costs 55 products instead of 100.

   Bounds (unsigned; every function states what it accepts):
     T "tight": limbs < 2^26+2^17 (even) / 2^25+2^17 (odd).  Output of
                fe_mul, fe_sqr, fe_wcarry, fe_unpack.
     L "loose": limbs < 1.5*2^27+2^17 (even) / 1.5*2^26+2^17 (odd).
                T+T, T+T+T, T-T (2p bias) and 2p-T are L.
   fe_mul/fe_sqr accept L inputs (every 32-bit operand, incl. 19*g and
   4*f, stays < 2^32 and every 64-bit column sum < 2^63).  fe_sub needs a
   T subtrahend.  Anything looser (e.g. L-L via fe_sub4) must go through
   fe_wcarry (one parallel carry step) before it reaches a multiply. */

#include <hip/hip_runtime.h>
#include <stdint.h>

#define FD_DEV __device__ __forceinline__

typedef uint32_t u32;
typedef uint64_t u64;
typedef int64_t  i64;

struct fe { u32 v[10]; };

FD_DEV u64 fd_mad( u32 a, u32 b, u64 c ) { return (u64)a * (u64)b + c; }

/* The same, with the result pinned behind an empty asm: the compiler may
   not re-associate a column chain (it would pull a non-zero initial
   accumulator -- a folded carry -- out into a separate 64-bit add). */
FD_DEV u64 fd_mad_a( u32 a, u32 b, u64 c ) {
  u64 r = (u64)a * (u64)b + c;
  asm( "" : "+v"( r ) );
  return r;
}


/* Scheduling fence after each multiply/square: keeps the machine
   scheduler from hoisting the next operation's operand preparation into
   this one's carry chain, which otherwise inflates register pressure
   several-fold on long dependent chains (pow22523: 256 -> ~110 VGPRs). */
#ifndef FD_SCHED_FENCE
#define FD_SCHED_FENCE() __builtin_amdgcn_sched_barrier( 0 )
#endif

#define FE_W(i)    ( ((i) & 1) ? 25 : 26 )
#define FE_M(i)    ( ((i) & 1) ? 0x1ffffffu : 0x3ffffffu )
#define FE_S(i)    ( (51*(i)+1) / 2 )            /* ceil(25.5 i) */

/* ---- constants ----------------------------------------------------- */

#define FE10(a0,a1,a2,a3,a4,a5,a6,a7,a8,a9) {{a0,a1,a2,a3,a4,a5,a6,a7,a8,a9}}

FD_DEV fe fe_zero( void ) { fe r = FE10(0,0,0,0,0,0,0,0,0,0); return r; }
FD_DEV fe fe_one ( void ) { fe r = FE10(1,0,0,0,0,0,0,0,0,0); return r; }
/* d = -121665/121666 */
FD_DEV fe fe_d( void )  { fe r = FE10(0x35978a3u,0x0d37284u,0x3156ebdu,0x06a0a0eu,0x001c029u,0x179e898u,0x3a03cbbu,0x1ce7198u,0x2e2b6ffu,0x1480db3u); return r; }
FD_DEV fe fe_d2( void ) { fe r = FE10(0x2b2f159u,0x1a6e509u,0x22add7au,0x0d4141du,0x0038052u,0x0f3d130u,0x3407977u,0x19ce331u,0x1c56dffu,0x0901b67u); return r; }
/* sqrt(-1) = 2^((p-1)/4) */
FD_DEV fe fe_sqrtm1( void ) { fe r = FE10(0x20ea0b0u,0x186c9d2u,0x08f189du,0x035697fu,0x0bd0c60u,0x1fbd7a7u,0x2804c9eu,0x1e16569u,0x004fc1du,0x0ae0c92u); return r; }
/* base point B (affine) */
FD_DEV fe fe_Bx( void ) { fe r = FE10(0x325d51au,0x18b5823u,0x0f6592au,0x104a92du,0x1a4b31du,0x1d6dc5cu,0x27118feu,0x07fd814u,0x13cd6e5u,0x085a4dbu); return r; }
FD_DEV fe fe_By( void ) { fe r = FE10(0x2666658u,0x1999999u,0x0ccccccu,0x1333333u,0x1999999u,0x0666666u,0x3333333u,0x0ccccccu,0x2666666u,0x1999999u); return r; }

/* y coordinates of the order-8 points (fd_curve25519.h:88-118), canonical 8x32 */
#define FD_Y0_W { 0x8f95e826u,0xb027b2c2u,0x89f4c345u,0xf098eff2u,0x05acdfd5u,0x3933c6d3u,0x880238b1u,0x05fc536du }
#define FD_Y1_W { 0x706a17c7u,0x4fd84d3du,0x760b3cbau,0x0f67100du,0xfa53202au,0xc6cc392cu,0x77fdc74eu,0x7a03ac92u }

/* ---- add / sub / carry ----------------------------------------------- */

/* r = a + b (no carry).  T+T -> L; (T+T)+T -> L. */
FD_DEV void fe_add( fe & r, fe const & a, fe const & b ) {
#pragma unroll
  for( int i=0; i<10; i++ ) r.v[i] = a.v[i] + b.v[i];
}

/* r = a - b + 2p.  b must be T (limbs <= 2p limbs).  a T -> r L. */
FD_DEV void fe_sub( fe & r, fe const & a, fe const & b ) {
#pragma unroll
  for( int i=0; i<10; i++ ) {
    u32 twop = (i==0) ? 0x7ffffdau : ( (i & 1) ? 0x3fffffeu : 0x7fffffeu );
    r.v[i] = a.v[i] + twop - b.v[i];
  }
}

/* r = a - b + 4p.  b may be L.  Result must be fe_wcarry'd before a mul. */
FD_DEV void fe_sub4( fe & r, fe const & a, fe const & b ) {
#pragma unroll
  for( int i=0; i<10; i++ ) {
    u32 fourp = (i==0) ? 0xfffffb4u : ( (i & 1) ? 0x7fffffcu : 0xffffffcu );
    r.v[i] = a.v[i] + fourp - b.v[i];
  }
}

/* r = -a = 2p - a (a T -> r L) */
FD_DEV void fe_neg( fe & r, fe const & a ) { fe z = fe_zero(); fe_sub( r, z, a ); }

/* one parallel carry step: limbs < 2^31 in -> T out */
FD_DEV void fe_wcarry( fe & r, fe const & a ) {
  u32 c[10];
#pragma unroll
  for( int i=0; i<10; i++ ) c[i] = a.v[i] >> FE_W(i);
  r.v[0] = (a.v[0] & FE_M(0)) + 19u * c[9];
#pragma unroll
  for( int i=1; i<10; i++ ) r.v[i] = (a.v[i] & FE_M(i)) + c[i-1];
}

/* 64-bit column sums -> T (carry order of ref10 fe_mul) */
FD_DEV void fe_carry64( fe & r, u64 h[ 10 ] ) {
  u64 c;
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
  c = h[9] >> 25; h[0] += c * 19u; h[9] &= 0x1ffffffUL;
  c = h[0] >> 26; h[1] += c; h[0] &= 0x3ffffffUL;
#pragma unroll
  for( int i=0; i<10; i++ ) r.v[i] = (u32)h[i];
}

/* ---- multiply / square ------------------------------------------------- */

/* Carry folding (FD_CARRY_FOLD=1): the columns are produced in two
   chains, 0..4 and 5..9, and each column's v_mad_u64_u32 chain starts
   from the carry out of the previous column, so the carry costs a shift
   and a mask but no 64-bit add (≈10 fewer VALU instructions per
   multiply).  The chains meet at limb 5 (carry out of 4) and limb 0
   (19 x carry out of 9), each a short second step.  Output T:
   r5 and r0 are re-masked, r6 and r1 take carries < 2^12 and < 2^15.

   The fold serialises each half's 50 multiplies through one accumulator:
   the fewest instructions, for kernels with waves enough per SIMD to hide
   the latency.  A kernel that runs one wave per SIMD (a batch of <= 64K
   signatures) finishes sooner with ten independent column chains (F = 0:
   more instructions, more VGPRs, 4x the ILP) -- profiles/r02/dsm_ab.  The
   multiply family below is templated on F; FD_CARRY_FOLD is the default. */
#ifndef FD_CARRY_FOLD
#define FD_CARRY_FOLD 1
#endif
template<int F> FD_DEV u64 fd_col_mad( u32 a, u32 b, u64 c ) {
  if constexpr( F != 0 ) return fd_mad_a( a, b, c );
  else                   return fd_mad( a, b, c );
}
#define FD_COL_MAD fd_col_mad<FM>
#define FE_FOLD_CHAINS( r, COL, ca, cb ) do {                               \
    _Pragma("unroll") for( int s_=0; s_<5; s_++ ) {                          \
      COL( s_, ca );     r.v[s_]   = (u32)ca & FE_M(s_);   ca >>= FE_W(s_);  \
      COL( s_+5, cb );   r.v[s_+5] = (u32)cb & FE_M(s_+5); cb >>= FE_W(s_+5);\
    }                                                                        \
    u64 t5_ = fd_add32( ca, r.v[5] );                                         \
    r.v[5] = (u32)t5_ & FE_M(5); r.v[6] += (u32)( t5_ >> 25 );                \
    u64 t0_ = (u64)r.v[0] + cb * 19u;                                        \
    r.v[0] = (u32)t0_ & FE_M(0); r.v[1] += (u32)( t0_ >> 26 );                \
  } while(0)

/* FD_FOLD4: four chains (columns 0-2, 3-4, 5-7, 8-9) instead of two: twice the independent
   accumulators, so consecutive multiply-adds of one chain are further apart (no wait state between
   them), for two more carry junctions (limbs 3 and 8).  A/B knob. */
#ifndef FD_FOLD4
#define FD_FOLD4 0
#endif
#define FE_FOLD_CHAINS4( r, COL, ca, cb ) do {                              \
    u64 cc = 0, cd = 0;                                                      \
    _Pragma("unroll") for( int t_=0; t_<3; t_++ ) {                          \
      COL( t_, ca );     r.v[t_]   = (u32)ca & FE_M(t_);   ca >>= FE_W(t_);  \
      if( t_ < 2 ) { COL( t_+3, cb ); r.v[t_+3] = (u32)cb & FE_M(t_+3); cb >>= FE_W(t_+3); } \
      COL( t_+5, cc );   r.v[t_+5] = (u32)cc & FE_M(t_+5); cc >>= FE_W(t_+5);\
      if( t_ < 2 ) { COL( t_+8, cd ); r.v[t_+8] = (u32)cd & FE_M(t_+8); cd >>= FE_W(t_+8); } \
    }                                                                        \
    u64 t3_ = fd_add32( ca, r.v[3] );                                        \
    r.v[3] = (u32)t3_ & FE_M(3); r.v[4] += (u32)( t3_ >> 25 );                \
    u64 t5_ = fd_add32( cb, r.v[5] );                                        \
    r.v[5] = (u32)t5_ & FE_M(5); r.v[6] += (u32)( t5_ >> 25 );                \
    u64 t8_ = fd_add32( cc, r.v[8] );                                        \
    r.v[8] = (u32)t8_ & FE_M(8); r.v[9] += (u32)( t8_ >> 26 );                \
    u64 t0_ = (u64)r.v[0] + cd * 19u;                                        \
    r.v[0] = (u32)t0_ & FE_M(0); r.v[1] += (u32)( t0_ >> 26 );                \
  } while(0)
#if FD_FOLD4
#undef  FE_FOLD_CHAINS
#define FE_FOLD_CHAINS FE_FOLD_CHAINS4
#endif

/* Operand multiples are formed only for the limbs that use them, each
   behind an empty asm so the compiler keeps one register per multiple
   instead of re-deriving it at every use (VALU-issue bound: every
   instruction counts). */
#define FD_KEEP( x ) asm( "" : "+v"( x ) )

/* 2x as x + x: on gfx950 v_add_u32 issues in 2.9 cycles per wave64 and
   v_lshlrev_b32 (what the compiler emits for 2x) in 4.75 (tools/instprobe,
   profiles/r02/roofline/instprobe.log); the asm also keeps the multiple in
   one register like FD_KEEP.  FD_ADD2=0: the compiler's shift. */
#ifndef FD_ADD2
#define FD_ADD2 1
#endif
FD_DEV u32 fd_x2( u32 x ) {
#if FD_ADD2
  u32 r; asm( "v_add_u32 %0, %1, %1" : "=v"( r ) : "v"( x ) ); return r;
#else
  u32 r = 2u * x; FD_KEEP( r ); return r;
#endif
}

/* acc + x for a 32-bit x.  FD_MAD1=1: as one v_mad_u64_u32 (x * 1 + acc, 4.66 cycles isolated)
   instead of zero-extending x (v_mov_b32) and a 64-bit add (v_lshl_add_u64, 7.5 cycles together).
   Off: the DSM's time follows its multiply-add count more than its other instructions (27 more
   v_mad_u64_u32 per doubling measured 0.3 % slower, four carry chains with ~14 more 2.5-4 % slower,
   profiles/r02/dsm_ab), so the add stays off the multiplier. */
#ifndef FD_MAD1
#define FD_MAD1 0
#endif
FD_DEV u64 fd_add32( u64 acc, u32 x ) {
#if FD_MAD1
  u64 r, cy;   /* (the compiler folds a C multiply by 1 back into the add: spell the instruction) */
  asm( "v_mad_u64_u32 %0, %1, %2, 1, %3" : "=v"( r ), "=s"( cy ) : "v"( x ), "v"( acc ) );
  return r;
#else
  return acc + (u64)x;
#endif
}

/* 19 g_j for j = 1..9 (the wrapped columns of a product with g) */
struct fe19 { u32 v[10]; };
FD_DEV void fe_x19( fe19 & r, fe const & g ) {
  r.v[0] = 0u;
#pragma unroll
  for( int j=1; j<10; j++ ) { r.v[j] = 19u * g.v[j]; FD_KEEP( r.v[j] ); }
}

/* r = f * g with g19 = fe_x19( g ) precomputed (shared by several
   products with the same g); f, g L -> r T.  Column k sums f_i g_j over
   i+j == k (mod 10); weight 2 when i and j are both odd
   (ceil(25.5i)+ceil(25.5j) = ceil(25.5(i+j)) + 1), weight 19 when
   i+j >= 10 (2^255 = 19).  100 v_mad_u64_u32 + 5 doublings. */
template<int FM = FD_CARRY_FOLD>
FD_DEV void fe_mul19( fe & r, fe const & f, fe const & g, fe19 const & g19 ) {
  u32 f2[10];
#pragma unroll
  for( int i=0; i<10; i++ ) { f2[i] = f.v[i]; if( i & 1 ) f2[i] = fd_x2( f.v[i] ); }
#define FE_MUL_COL( k, acc ) do {                                      \
    _Pragma("unroll") for( int i=0; i<10; i++ ) {                       \
      int j = (k) - i, wrap = j < 0;                                    \
      if( wrap ) j += 10;                                               \
      u32 a_ = ( (i & 1) && (j & 1) ) ? f2[i] : f.v[i];                 \
      u32 b_ = wrap ? g19.v[j] : g.v[j];                                \
      acc = FD_COL_MAD( a_, b_, acc );                                  \
    } } while(0)
  if constexpr( FM != 0 ) {
    u64 ca = 0, cb = 0; fe o;   /* o: r may alias f or g */
    FE_FOLD_CHAINS( o, FE_MUL_COL, ca, cb );
    r = o;
  } else {
    u64 h[10];
#pragma unroll
    for( int k=0; k<10; k++ ) { u64 acc = 0; FE_MUL_COL( k, acc ); h[k] = acc; }
    fe_carry64( r, h );
  }
#undef FE_MUL_COL
  FD_SCHED_FENCE();
}

template<int FM = FD_CARRY_FOLD>
FD_DEV void fe_mul( fe & r, fe const & f, fe const & g ) {
  fe19 g19; fe_x19( g19, g );
  fe_mul19<FM>( r, f, g, g19 );
}

/* r = f^2; f L -> r T.  55 products; coefficient c = (i<j ? 2 : 1) x
   (i, j both odd ? 2 : 1) x (i+j >= 10 ? 19 : 1) is carried by the
   operands f, 2f (i<=8), 38f (odd j>=5) and 19f (even j>=6) -- 14
   multiples.  Largest operand 38f_odd < 2^31.9 (L input). */
#define FE_SQR_OPERANDS( f )                                                  \
  u32 f2[10], fw[10];                                                         \
  _Pragma("unroll") for( int i=0; i<9; i++ ) f2[i] = fd_x2( f.v[i] );          \
  f2[9] = 0u;                                                                 \
  _Pragma("unroll") for( int j=0; j<10; j++ ) {                               \
    fw[j] = 0u;                                                               \
    if( j >= 5 ) { fw[j] = ( (j & 1) ? 38u : 19u ) * f.v[j]; FD_KEEP( fw[j] ); } \
  }
#define FE_SQR_COL( k, acc ) do {                                             \
    _Pragma("unroll") for( int i=0; i<10; i++ ) {                              \
      _Pragma("unroll") for( int j=i; j<10; j++ ) {                            \
        if( ( (i + j) % 10 ) != (k) ) continue;                                \
        int odd2 = (i & 1) && (j & 1);                                         \
        int pair = i < j;                                                      \
        int wrap = i + j >= 10;                                                \
        u32 a_, b_;                                                            \
        if( !wrap ) {                                                          \
          int c = (pair ? 2 : 1) * (odd2 ? 2 : 1);                             \
          a_ = c==1 ? f.v[i] : f2[i];                                          \
          b_ = c==4 ? f2[j]  : f.v[j];                                         \
        } else if( j & 1 ) {  /* b = 38 f_j: c/38 = 1/2 (i==j), 1, 2 */        \
          int c2 = (pair ? 2 : 1) * (odd2 ? 2 : 1);                            \
          a_ = c2==4 ? f2[i] : f.v[i];                                         \
          b_ = fw[j];                                                          \
        } else {              /* even j: b = 19 f_j, c/19 = 1 (i==j) or 2 */   \
          a_ = pair ? f2[i] : f.v[i];                                          \
          b_ = fw[j];                                                          \
        }                                                                      \
        acc = FD_COL_MAD( a_, b_, acc );                                       \
      }                                                                        \
    } } while(0)

/* r = f^2; f L -> r T.  55 products; coefficient c = (i<j ? 2 : 1) x
   (i, j both odd ? 2 : 1) x (i+j >= 10 ? 19 : 1) is carried by the
   operands f, 2f (i<=8), 38f (odd j>=5) and 19f (even j>=6) -- 14
   multiples.  Largest operand 38f_odd < 2^31.9 (L input). */
template<int FM = FD_CARRY_FOLD>
FD_DEV void fe_sqr( fe & r, fe const & f ) {
  FE_SQR_OPERANDS( f );
  if constexpr( FM != 0 ) {
    u64 ca = 0, cb = 0; fe o;
    FE_FOLD_CHAINS( o, FE_SQR_COL, ca, cb );
    r = o;
  } else {
    u64 h[10];
#pragma unroll
    for( int k=0; k<10; k++ ) { u64 acc = 0; FE_SQR_COL( k, acc ); h[k] = acc; }
    fe_carry64( r, h );
  }
  FD_SCHED_FENCE();
}

/* 4p limbs: a bias larger than any L limb, for subtractions folded into
   the column sums of a square before its carry chain */
#define FE_4P(i) ( (i)==0 ? 0xfffffb4u : ( ((i) & 1) ? 0x7fffffcu : 0xffffffcu ) )

/* r = f^2 + 4p - b (b L) -> T: the subtraction rides on the squaring's
   carry chain instead of a separate biased sub + fe_wcarry */
template<int FM = FD_CARRY_FOLD>
FD_DEV void fe_sqr_sub( fe & r, fe const & f, fe const & b ) {
  FE_SQR_OPERANDS( f );
  if constexpr( FM != 0 ) {
#define FE_SQR_SUB_COL( k, acc ) do { acc = fd_add32( acc, FE_4P(k) - b.v[k] ); FE_SQR_COL( k, acc ); } while(0)
    u64 ca = 0, cb = 0; fe o;
    FE_FOLD_CHAINS( o, FE_SQR_SUB_COL, ca, cb );
    r = o;
#undef FE_SQR_SUB_COL
  } else {
    u64 h[10];
#pragma unroll
    for( int k=0; k<10; k++ ) { u64 acc = (u64)( FE_4P(k) - b.v[k] ); FE_SQR_COL( k, acc ); h[k] = acc; }
    fe_carry64( r, h );
  }
  FD_SCHED_FENCE();
}

/* r = 2 f^2 + 4p - b (b L) -> T.  FD_SQR2_PRE: f must be T (every caller
   passes a point's Z straight from a multiply); the factor 2 rides in the
   operands -- multiples f, 2f, 4f (limbs 1, 3), 38f (even j >= 6) and 76f
   (odd j >= 5), all < 2^31.3 for T limbs -- so each column accumulates into
   the carry chain directly instead of a separate sum doubled into it
   (v_lshl_add_u64 per column).  Column sums stay < 2^62. */
#ifndef FD_SQR2_PRE
#define FD_SQR2_PRE 1
#endif
#define FE_SQR2_OPERANDS( f )                                                 \
  u32 g2[10], g4[4], gw[10];                                                  \
  _Pragma("unroll") for( int i=0; i<10; i++ ) g2[i] = fd_x2( f.v[i] );        \
  g4[0] = g4[2] = 0u; g4[1] = fd_x2( g2[1] ); g4[3] = fd_x2( g2[3] );         \
  _Pragma("unroll") for( int j=0; j<10; j++ ) {                               \
    gw[j] = 0u;                                                               \
    if( j >= 5 ) { gw[j] = ( (j & 1) ? 76u : 38u ) * f.v[j]; FD_KEEP( gw[j] ); } \
  }
#define FE_SQR2_COL( k, acc ) do {                                            \
    _Pragma("unroll") for( int i=0; i<10; i++ ) {                              \
      _Pragma("unroll") for( int j=i; j<10; j++ ) {                            \
        if( ( (i + j) % 10 ) != (k) ) continue;                                \
        int odd2 = (i & 1) && (j & 1);                                         \
        int pair = i < j;                                                      \
        int wrap = i + j >= 10;                                                \
        u32 a_, b_;                                                            \
        if( !wrap ) {         /* 2c = 2, 4 or 8 */                             \
          int c = 2 * (pair ? 2 : 1) * (odd2 ? 2 : 1);                         \
          a_ = c==8 ? g4[i & 3] : g2[i];                                       \
          b_ = c==2 ? f.v[j] : g2[j];                                          \
        } else if( j & 1 ) {  /* b = 76 f_j: 2c/76 = 1 or 2 */                 \
          a_ = ( pair && odd2 ) ? g2[i] : f.v[i];                              \
          b_ = gw[j];                                                          \
        } else {              /* b = 38 f_j: 2c/38 = 1 (i == j) or 2 */        \
          a_ = pair ? g2[i] : f.v[i];                                          \
          b_ = gw[j];                                                          \
        }                                                                      \
        acc = FD_COL_MAD( a_, b_, acc );                                       \
      }                                                                        \
    } } while(0)

template<int FM = FD_CARRY_FOLD>
FD_DEV void fe_sqr2_sub( fe & r, fe const & f, fe const & b ) {
#if FD_SQR2_PRE
  FE_SQR2_OPERANDS( f );
  if constexpr( FM != 0 ) {
#define FE_SQR2P_SUB_COL( k, acc ) do { acc = fd_add32( acc, FE_4P(k) - b.v[k] ); FE_SQR2_COL( k, acc ); } while(0)
    u64 ca = 0, cb = 0; fe o;
    FE_FOLD_CHAINS( o, FE_SQR2P_SUB_COL, ca, cb );
    r = o;
#undef FE_SQR2P_SUB_COL
  } else {
    u64 h[10];
#pragma unroll
    for( int k=0; k<10; k++ ) { u64 acc = (u64)( FE_4P(k) - b.v[k] ); FE_SQR2_COL( k, acc ); h[k] = acc; }
    fe_carry64( r, h );
  }
#else
  FE_SQR_OPERANDS( f );
  if constexpr( FM != 0 ) {
#define FE_SQR2_SUB_COL( k, acc ) do { u64 h_ = 0; FE_SQR_COL( k, h_ ); acc = ( h_ << 1 ) + acc + (u64)( FE_4P(k) - b.v[k] ); } while(0)
    u64 ca = 0, cb = 0; fe o;
    FE_FOLD_CHAINS( o, FE_SQR2_SUB_COL, ca, cb );
    r = o;
#undef FE_SQR2_SUB_COL
  } else {
    u64 h[10];
#pragma unroll
    for( int k=0; k<10; k++ ) { u64 acc = 0; FE_SQR_COL( k, acc ); h[k] = ( acc << 1 ) + (u64)( FE_4P(k) - b.v[k] ); }
    fe_carry64( r, h );
  }
#endif
  FD_SCHED_FENCE();
}

/* r = a^(2^n) */
template<int FM = FD_CARRY_FOLD>
FD_DEV void fe_sqrn( fe & r, fe const & a, int n ) {
  fe_sqr<FM>( r, a );
#pragma unroll 1
  for( int i=1; i<n; i++ ) fe_sqr<FM>( r, r );
}

/* ---- packed 8 x 32-bit form (canonical) ---------------------------------- */

/* w (8 LE words, bit 255 ignored) -> limbs (T); accepts non-canonical
   values >= p (fd_f25519_frombytes / fiat curve25519_64.c:802) */
FD_DEV void fe_unpack( fe & r, u32 const w[ 8 ] ) {
#pragma unroll
  for( int i=0; i<10; i++ ) {
    int s = FE_S(i), wi = s >> 5, sh = s & 31;
    u32 lo = w[wi], hi = wi+1 < 8 ? w[wi+1] : 0u;
    r.v[i] = __builtin_amdgcn_alignbit( hi, lo, (u32)sh ) & FE_M(i);
  }
}

/* canonical value in [0,p) as 8 LE words; input limbs < 2^31 */
FD_DEV void fe_pack( u32 w[ 8 ], fe const & a ) {
  u32 h[10];
#pragma unroll
  for( int i=0; i<10; i++ ) h[i] = a.v[i];
  /* one carry pass: limbs 1-9 exact, h0 < 2^26 + 19 * 65, so h < 2^255 + 2^11 < 2p and the
     quotient ripple below sees carries of 0 or 1 (a second pass here changed nothing: checked on
     limbs up to 2^31 - 1 and on values around p, 2p and 2^255, against the value mod p) */
#pragma unroll
  for( int i=0; i<9; i++ ) { h[i+1] += h[i] >> FE_W(i); h[i] &= FE_M(i); }
  h[0] += 19u * (h[9] >> 25); h[9] &= 0x1ffffffu;
  /* subtract p iff h + 19 >= 2^255 */
  u32 q = (h[0] + 19u) >> 26;
#pragma unroll
  for( int i=1; i<10; i++ ) q = (h[i] + q) >> FE_W(i);
  h[0] += 19u * q;
#pragma unroll
  for( int i=0; i<9; i++ ) { h[i+1] += h[i] >> FE_W(i); h[i] &= FE_M(i); }
  h[9] &= 0x1ffffffu;
#pragma unroll
  for( int k=0; k<8; k++ ) w[k] = 0u;
#pragma unroll
  for( int i=0; i<10; i++ ) {
    int s = FE_S(i), wi = s >> 5, sh = s & 31;
    w[wi] |= h[i] << sh;
    if( sh + FE_W(i) > 32 && wi+1 < 8 ) w[wi+1] |= h[i] >> (32 - sh);
  }
}

FD_DEV int fe_is_zero( fe const & a ) {
  u32 w[8]; fe_pack( w, a );
  u32 o = 0;
#pragma unroll
  for( int i=0; i<8; i++ ) o |= w[i];
  return o==0u;
}

/* a == b (a, b L at most) */
FD_DEV int fe_eq( fe const & a, fe const & b ) { fe d; fe_sub4( d, a, b ); return fe_is_zero( d ); }

FD_DEV int fe_eq_words( fe const & a, u32 const w[ 8 ] ) {
  u32 x[8]; fe_pack( x, a );
  u32 o = 0;
#pragma unroll
  for( int i=0; i<8; i++ ) o |= x[i] ^ w[i];
  return o==0u;
}

/* parity of the canonical value ("sign" of x, RFC 8032) */
FD_DEV int fe_is_odd( fe const & a ) { u32 w[8]; fe_pack( w, a ); return (int)(w[0] & 1u); }

FD_DEV void fe_sel( fe & r, int c, fe const & a, fe const & b ) { /* r = c ? a : b */
#pragma unroll
  for( int i=0; i<10; i++ ) r.v[i] = c ? a.v[i] : b.v[i];
}

/* ---- exponentiations ------------------------------------------------------ */

/* r = a^(2^252-3): the addition chain of fd_f25519_pow22523
   (src/ballet/ed25519/fd_f25519.c:10-59). */
template<int FM = FD_CARRY_FOLD>
FD_DEV void fe_pow22523( fe & r, fe const & a ) {
  fe t0, t1, t2;
  fe_sqr<FM>( t0, a );
  fe_sqrn<FM>( t1, t0, 2 );
  fe_mul<FM>( t1, a, t1 );
  fe_mul<FM>( t0, t0, t1 );
  fe_sqr<FM>( t0, t0 );
  fe_mul<FM>( t0, t1, t0 );
  fe_sqrn<FM>( t1, t0, 5 );
  fe_mul<FM>( t0, t1, t0 );
  fe_sqrn<FM>( t1, t0, 10 );
  fe_mul<FM>( t1, t1, t0 );
  fe_sqrn<FM>( t2, t1, 20 );
  fe_mul<FM>( t1, t2, t1 );
  fe_sqrn<FM>( t1, t1, 10 );
  fe_mul<FM>( t0, t1, t0 );
  fe_sqrn<FM>( t1, t0, 50 );
  fe_mul<FM>( t1, t1, t0 );
  fe_sqrn<FM>( t2, t1, 100 );
  fe_mul<FM>( t1, t2, t1 );
  fe_sqrn<FM>( t1, t1, 50 );
  fe_mul<FM>( t0, t1, t0 );
  fe_sqrn<FM>( t0, t0, 2 );
  fe_mul<FM>( r, t0, a );
}

/* r = a^(p-2) = a^-1: the addition chain of fd_f25519_inv
   (src/ballet/ed25519/fd_f25519.c:62-103).  Off the hot path. */
template<int FM = FD_CARRY_FOLD>
FD_DEV void fe_invert( fe & r, fe const & z ) {
  fe t0, t1, t2, t3;
  fe_sqr<FM>( t0, z );
  fe_sqrn<FM>( t1, t0, 2 );
  fe_mul<FM>( t1, z, t1 );
  fe_mul<FM>( t0, t0, t1 );
  fe_sqr<FM>( t2, t0 );
  fe_mul<FM>( t1, t1, t2 );
  fe_sqrn<FM>( t2, t1, 5 );   fe_mul<FM>( t1, t2, t1 );
  fe_sqrn<FM>( t2, t1, 10 );  fe_mul<FM>( t2, t2, t1 );
  fe_sqrn<FM>( t3, t2, 20 );  fe_mul<FM>( t2, t3, t2 );
  fe_sqrn<FM>( t2, t2, 10 );  fe_mul<FM>( t1, t2, t1 );
  fe_sqrn<FM>( t2, t1, 50 );  fe_mul<FM>( t2, t2, t1 );
  fe_sqrn<FM>( t3, t2, 100 ); fe_mul<FM>( t2, t3, t2 );
  fe_sqrn<FM>( t2, t2, 50 );  fe_mul<FM>( t1, t2, t1 );
  fe_sqrn<FM>( t1, t1, 5 );
  fe_mul<FM>( r, t1, t0 );
}
