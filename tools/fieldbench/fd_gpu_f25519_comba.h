#pragma once
/* fd_gpu_f25519.h -- GF(2^255-19) for CDNA4 (gfx950), one field element
   per lane in 8 x 32-bit limbs (little endian), device code only.

   MI355X-native replacement for the reference's field layer
   (src/ballet/ed25519/fd_f25519.h API; AVX-512 r43x6 backend
   avx512/fd_r43x6.h, portable fiat 5x51 backend ref/fd_f25519.h).  Not a
   port of either: the reference packs ONE element into 6 lanes of a zmm
   (latency-optimised, one signature at a time); here each of the 64
   lanes of a wave owns a whole element of its own signature, and the
   limb products are v_mad_u64_u32 (32x32+64 -> 64, carry-out in an SGPR
   pair) carry chains.

   Representation invariant: a "fe" holds any value in [0, 2^256) that is
   congruent to the field element (weakly reduced); fe_canon() maps to
   [0,p).  Every operation below accepts and returns weakly reduced
   values, so there is no overflow bookkeeping between operations. */

#include <hip/hip_runtime.h>
#include <stdint.h>

#define FD_DEV __device__ __forceinline__

typedef uint32_t u32;
typedef uint64_t u64;
typedef int64_t  i64;

struct fe { u32 v[8]; };

FD_DEV u64 fd_mad( u32 a, u32 b, u64 c ) { return (u64)a * (u64)b + c; }

/* ---- constants ----------------------------------------------------- */

#define FE_C(a0,a1,a2,a3,a4,a5,a6,a7) {{a0,a1,a2,a3,a4,a5,a6,a7}}

FD_DEV fe fe_zero( void ) { fe r = FE_C(0,0,0,0,0,0,0,0); return r; }
FD_DEV fe fe_one ( void ) { fe r = FE_C(1,0,0,0,0,0,0,0); return r; }
/* d = -121665/121666 */
FD_DEV fe fe_d   ( void ) { fe r = FE_C(0x135978a3u,0x75eb4dcau,0x4141d8abu,0x00700a4du,0x7779e898u,0x8cc74079u,0x2b6ffe73u,0x52036ceeu); return r; }
FD_DEV fe fe_d2  ( void ) { fe r = FE_C(0x26b2f159u,0xebd69b94u,0x8283b156u,0x00e0149au,0xeef3d130u,0x198e80f2u,0x56dffce7u,0x2406d9dcu); return r; }
/* sqrt(-1) = 2^((p-1)/4) */
FD_DEV fe fe_sqrtm1( void ) { fe r = FE_C(0x4a0ea0b0u,0xc4ee1b27u,0xad2fe478u,0x2f431806u,0x3dfbd7a7u,0x2b4d0099u,0x4fc1df0bu,0x2b832480u); return r; }
/* y coordinates of the order-8 points (fd_curve25519.h:88-118) */
FD_DEV fe fe_y0  ( void ) { fe r = FE_C(0x8f95e826u,0xb027b2c2u,0x89f4c345u,0xf098eff2u,0x05acdfd5u,0x3933c6d3u,0x880238b1u,0x05fc536du); return r; }
FD_DEV fe fe_y1  ( void ) { fe r = FE_C(0x706a17c7u,0x4fd84d3du,0x760b3cbau,0x0f67100du,0xfa53202au,0xc6cc392cu,0x77fdc74eu,0x7a03ac92u); return r; }
/* base point B (affine) */
FD_DEV fe fe_Bx  ( void ) { fe r = FE_C(0x8f25d51au,0xc9562d60u,0x9525a7b2u,0x692cc760u,0xfdd6dc5cu,0xc0a4e231u,0xcd6e53feu,0x216936d3u); return r; }
FD_DEV fe fe_By  ( void ) { fe r = FE_C(0x66666658u,0x66666666u,0x66666666u,0x66666666u,0x66666666u,0x66666666u,0x66666666u,0x66666666u); return r; }

/* ---- add / sub ----------------------------------------------------- */

/* r = a + b mod p (weak).  a+b < 2^257: fold the carry as 38 (2^256 = 38
   mod p); a second carry is only possible when the low 256 bits are
   < 38, so the final 38*c cannot overflow. */
FD_DEV void fe_add( fe & r, fe const & a, fe const & b ) {
  u64 c = 0;
#pragma unroll
  for( int i=0; i<8; i++ ) { c += (u64)a.v[i] + (u64)b.v[i]; r.v[i] = (u32)c; c >>= 32; }
  c *= 38u;
#pragma unroll
  for( int i=0; i<8; i++ ) { c += (u64)r.v[i]; r.v[i] = (u32)c; c >>= 32; }
  r.v[0] += (u32)c * 38u;
}

/* r = a - b mod p (weak).  A borrow means the result wrapped by 2^256
   = 38 mod p, so subtract 38; a second borrow (low part < 38) wraps
   again and is fixed by one more -38 that cannot borrow. */
FD_DEV void fe_sub( fe & r, fe const & a, fe const & b ) {
  u64 c = 0;
#pragma unroll
  for( int i=0; i<8; i++ ) { c = (u64)a.v[i] - (u64)b.v[i] - c; r.v[i] = (u32)c; c = (c >> 32) & 1u; }
  c *= 38u;
#pragma unroll
  for( int i=0; i<8; i++ ) { c = (u64)r.v[i] - c; r.v[i] = (u32)c; c = (c >> 32) & 1u; }
  r.v[0] -= (u32)c * 38u;
}

FD_DEV void fe_neg( fe & r, fe const & a ) { fe z = fe_zero(); fe_sub( r, z, a ); }

/* ---- 256x256 -> 512 products and the 512 -> 256 fold -------------- */

/* r = t mod p (weak), t = 16 words.  2^256 = 38 mod p. */
FD_DEV void fe_fold512( fe & r, u32 const t[ 16 ] ) {
  u64 c = 0;
#pragma unroll
  for( int i=0; i<8; i++ ) { c = fd_mad( t[8+i], 38u, c + (u64)t[i] ); r.v[i] = (u32)c; c >>= 32; }
  c *= 38u;                         /* c <= 38 -> <= 1444 */
#pragma unroll
  for( int i=0; i<8; i++ ) { c += (u64)r.v[i]; r.v[i] = (u32)c; c >>= 32; }
  r.v[0] += (u32)c * 38u;
}

#ifndef FD_GPU_MUL_ASM
#define FD_GPU_MUL_ASM 1
#endif

#if FD_GPU_MUL_ASM
/* Product scanning (Comba) with a 96-bit column accumulator {acc64,hi}:
   v_mad_u64_u32 acc = a*b + acc (carry-out -> SGPR pair), then
   v_addc_co_u32 hi += carry.  Two VALU ops per 32x32 product. */
FD_DEV void fd_mac( u64 & acc, u32 & hi, u32 a, u32 b ) {
  u64 cc;
  asm( "v_mad_u64_u32 %0, %2, %3, %4, %0\n\t"
                "v_addc_co_u32_e64 %1, %2, %1, 0, %2"
                : "+v"(acc), "+v"(hi), "=&s"(cc)
                : "v"(a), "v"(b) );
}
/* first product of a column whose running accumulator is {acc64} only */
FD_DEV void fd_mac0( u64 & acc, u32 & hi, u32 a, u32 b ) {
  u64 cc;
  asm( "v_mad_u64_u32 %0, %2, %3, %4, %0\n\t"
                "v_addc_co_u32_e64 %1, %2, 0, 0, %2"
                : "+v"(acc), "=v"(hi), "=&s"(cc)
                : "v"(a), "v"(b) );
}

FD_DEV void fe_mul_wide( u32 t[ 16 ], fe const & a, fe const & b ) {
  u64 acc = 0; u32 hi = 0;
#pragma unroll
  for( int k=0; k<15; k++ ) {
    int first = 1;
#pragma unroll
    for( int i=0; i<8; i++ ) {
      int j = k - i;
      if( j<0 || j>7 ) continue;
      if( first ) { fd_mac0( acc, hi, a.v[i], b.v[j] ); first = 0; }
      else          fd_mac ( acc, hi, a.v[i], b.v[j] );
    }
    t[k] = (u32)acc;
    acc  = (acc >> 32) | ((u64)hi << 32);
  }
  t[15] = (u32)acc;
}

/* squaring: cross products once, doubled, plus the diagonal */
FD_DEV void fe_sqr_wide( u32 t[ 16 ], fe const & a ) {
  u64 acc = 0; u32 hi = 0;
#pragma unroll
  for( int k=0; k<15; k++ ) {
    /* column k: sum_{i<j, i+j=k} a_i a_j, doubled, + a_{k/2}^2 */
    u64 x = 0; u32 xh = 0; int first = 1;
#pragma unroll
    for( int i=0; i<8; i++ ) {
      int j = k - i;
      if( j<=i || j>7 ) continue;
      if( first ) { fd_mac0( x, xh, a.v[i], a.v[j] ); first = 0; }
      else          fd_mac ( x, xh, a.v[i], a.v[j] );
    }
    /* acc += 2*x */
    u64 x2 = x << 1; u32 x2h = (xh << 1) | (u32)(x >> 63);
    if( first ) { x2 = 0; x2h = 0; }
    if( !(k & 1) ) { u32 d = a.v[k>>1]; u64 sq = (u64)d * d; u64 s = x2 + sq; x2h += (s < x2); x2 = s; }
    u64 s = acc + x2; u32 carry = (s < acc);
    acc = s; hi += x2h + carry;
    t[k] = (u32)acc;
    acc  = (acc >> 32) | ((u64)hi << 32);
    hi = 0;
  }
  t[15] = (u32)acc;
}
#else
/* Operand scanning in plain C (compiler picks v_mad_u64_u32). */
FD_DEV void fe_mul_wide( u32 t[ 16 ], fe const & a, fe const & b ) {
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
}
FD_DEV void fe_sqr_wide( u32 t[ 16 ], fe const & a ) { fe_mul_wide( t, a, a ); }
#endif

FD_DEV void fe_mul( fe & r, fe const & a, fe const & b ) { u32 t[16]; fe_mul_wide( t, a, b ); fe_fold512( r, t ); }
FD_DEV void fe_sqr( fe & r, fe const & a ) { u32 t[16]; fe_sqr_wide( t, a ); fe_fold512( r, t ); }

/* r = a^(2^n) */
FD_DEV void fe_sqrn( fe & r, fe const & a, int n ) {
  fe_sqr( r, a );
#pragma unroll 1
  for( int i=1; i<n; i++ ) fe_sqr( r, r );
}

/* ---- canonical form and comparisons -------------------------------- */

/* r = a mod p in [0,p) */
FD_DEV void fe_canon( fe & r, fe const & a ) {
  /* fold bit 255: a = h*2^255 + l, 2^255 = 19 mod p */
  u32 h = a.v[7] >> 31;
  u64 c = (u64)h * 19u;
#pragma unroll
  for( int i=0; i<8; i++ ) { c += (u64)( i==7 ? (a.v[7] & 0x7fffffffu) : a.v[i] ); r.v[i] = (u32)c; c >>= 32; }
  /* now r < 2^255 + 19; r >= p  <=>  r + 19 >= 2^255 */
  u32 t[8]; c = 19;
#pragma unroll
  for( int i=0; i<8; i++ ) { c += (u64)r.v[i]; t[i] = (u32)c; c >>= 32; }
  u32 ge = t[7] >> 31;
#pragma unroll
  for( int i=0; i<8; i++ ) r.v[i] = ge ? t[i] : r.v[i];
  r.v[7] &= ge ? 0x7fffffffu : 0xffffffffu;
}

FD_DEV int fe_is_zero( fe const & a ) {
  fe c; fe_canon( c, a );
  u32 o = 0;
#pragma unroll
  for( int i=0; i<8; i++ ) o |= c.v[i];
  return o==0u;
}

FD_DEV int fe_eq( fe const & a, fe const & b ) { fe d; fe_sub( d, a, b ); return fe_is_zero( d ); }

/* parity of the canonical value ("sign" of x, RFC 8032) */
FD_DEV int fe_is_odd( fe const & a ) { fe c; fe_canon( c, a ); return (int)(c.v[0] & 1u); }

FD_DEV void fe_sel( fe & r, int c, fe const & a, fe const & b ) { /* r = c ? a : b */
#pragma unroll
  for( int i=0; i<8; i++ ) r.v[i] = c ? a.v[i] : b.v[i];
}

/* r = a^(2^252-3): the addition chain of fd_f25519_pow22523
   (src/ballet/ed25519/fd_f25519.c:10-59). */
FD_DEV void fe_pow22523( fe & r, fe const & a ) {
  fe t0, t1, t2;
  fe_sqr ( t0, a );
  fe_sqrn( t1, t0, 2 );
  fe_mul ( t1, a, t1 );
  fe_mul ( t0, t0, t1 );
  fe_sqr ( t0, t0 );
  fe_mul ( t0, t1, t0 );
  fe_sqrn( t1, t0, 5 );
  fe_mul ( t0, t1, t0 );
  fe_sqrn( t1, t0, 10 );
  fe_mul ( t1, t1, t0 );
  fe_sqrn( t2, t1, 20 );
  fe_mul ( t1, t2, t1 );
  fe_sqrn( t1, t1, 10 );
  fe_mul ( t0, t1, t0 );
  fe_sqrn( t1, t0, 50 );
  fe_mul ( t1, t1, t0 );
  fe_sqrn( t2, t1, 100 );
  fe_mul ( t1, t2, t1 );
  fe_sqrn( t1, t1, 50 );
  fe_mul ( t0, t1, t0 );
  fe_sqrn( t0, t0, 2 );
  fe_mul ( r, t0, a );
}

/* r = a^(p-2) = a^-1: the addition chain of fd_f25519_inv
   (src/ballet/ed25519/fd_f25519.c:62-103).  Only used off the hot path
   (base-table setup). */
FD_DEV void fe_invert( fe & r, fe const & z ) {
  fe t0, t1, t2, t3;
  fe_sqr ( t0, z );
  fe_sqrn( t1, t0, 2 );
  fe_mul ( t1, z, t1 );
  fe_mul ( t0, t0, t1 );
  fe_sqr ( t2, t0 );
  fe_mul ( t1, t1, t2 );
  fe_sqrn( t2, t1, 5 );   fe_mul( t1, t2, t1 );
  fe_sqrn( t2, t1, 10 );  fe_mul( t2, t2, t1 );
  fe_sqrn( t3, t2, 20 );  fe_mul( t2, t3, t2 );
  fe_sqrn( t2, t2, 10 );  fe_mul( t1, t2, t1 );
  fe_sqrn( t2, t1, 50 );  fe_mul( t2, t2, t1 );
  fe_sqrn( t3, t2, 100 ); fe_mul( t2, t3, t2 );
  fe_sqrn( t2, t2, 50 );  fe_mul( t1, t2, t1 );
  fe_sqrn( t1, t1, 5 );
  fe_mul ( r, t1, t0 );
}

/* Two independent pow22523 chains interleaved (decode of A and R at
   once, the GPU analogue of FD_R43X6_POW22523_2_INL): the two chains give
   the scheduler independent v_mad_u64_u32 streams to overlap. */
FD_DEV void fe_sqrn2( fe & r, fe const & a, fe & s, fe const & b, int n ) {
  fe_sqr( r, a ); fe_sqr( s, b );
#pragma unroll 1
  for( int i=1; i<n; i++ ) { fe_sqr( r, r ); fe_sqr( s, s ); }
}

FD_DEV void fe_pow22523_2( fe & r, fe const & a, fe & s, fe const & b ) {
  fe t0, t1, t2, u0, u1, u2;
  fe_sqr ( t0, a );              fe_sqr ( u0, b );
  fe_sqrn2( t1, t0, u1, u0, 2 );
  fe_mul ( t1, a, t1 );          fe_mul ( u1, b, u1 );
  fe_mul ( t0, t0, t1 );         fe_mul ( u0, u0, u1 );
  fe_sqr ( t0, t0 );             fe_sqr ( u0, u0 );
  fe_mul ( t0, t1, t0 );         fe_mul ( u0, u1, u0 );
  fe_sqrn2( t1, t0, u1, u0, 5 );
  fe_mul ( t0, t1, t0 );         fe_mul ( u0, u1, u0 );
  fe_sqrn2( t1, t0, u1, u0, 10 );
  fe_mul ( t1, t1, t0 );         fe_mul ( u1, u1, u0 );
  fe_sqrn2( t2, t1, u2, u1, 20 );
  fe_mul ( t1, t2, t1 );         fe_mul ( u1, u2, u1 );
  fe_sqrn2( t1, t1, u1, u1, 10 );
  fe_mul ( t0, t1, t0 );         fe_mul ( u0, u1, u0 );
  fe_sqrn2( t1, t0, u1, u0, 50 );
  fe_mul ( t1, t1, t0 );         fe_mul ( u1, u1, u0 );
  fe_sqrn2( t2, t1, u2, u1, 100 );
  fe_mul ( t1, t2, t1 );         fe_mul ( u1, u2, u1 );
  fe_sqrn2( t1, t1, u1, u1, 50 );
  fe_mul ( t0, t1, t0 );         fe_mul ( u0, u1, u0 );
  fe_sqrn2( t0, t0, u0, u0, 2 );
  fe_mul ( r, t0, a );           fe_mul ( s, u0, b );
}

/* ---- byte <-> limb -------------------------------------------------- */

/* limbs from 8 little-endian words, bit 255 dropped (non-canonical y >= p
   accepted as in fd_f25519_frombytes / fiat curve25519_64.c:802) */
FD_DEV void fe_from_words( fe & r, u32 const w[ 8 ] ) {
#pragma unroll
  for( int i=0; i<8; i++ ) r.v[i] = w[i];
  r.v[7] &= 0x7fffffffu;
}
