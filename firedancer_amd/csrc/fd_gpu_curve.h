#pragma once
/* fd_gpu_curve.h -- edwards25519 group and scalar layer, CDNA4 device code.

   Replaces the reference's curve/scalar layer on the verify path:
   point decompression (fd_ed25519_point_frombytes_2x ->
   FD_R43X6_GE_DECODE2, avx512/fd_r43x6_ge.c:163-254), small-order test
   (fd_ed25519_affine_is_small_order, fd_curve25519.h:88-118), extended
   coordinate dbl/add (FD_R43X6_GE_DBL/ADD, avx512/fd_r43x6_ge.h:119-236),
   scalar validate/reduce (fd_curve25519_scalar.h:57-73,
   fd_curve25519_scalar.c:3-110).  One signature per lane. */

#include "fd_gpu_f25519.h"

struct ge_p2    { fe X, Y, Z; };        /* projective                    */
struct ge_p3    { fe X, Y, Z, T; };     /* extended, T = XY/Z            */
struct ge_p1p1  { fe X, Y, Z, T; };     /* completed: (X:T),(Y:Z)        */
struct ge_cached{ fe YpX, YmX, Z, T2d; };
struct ge_precomp{ fe ypx, ymx, xy2d; };/* affine, Z = 1                 */

/* Bound annotations (fd_gpu_f25519.h): every coordinate handed to a
   multiply is T or L; the two "D-C"/"E" style differences of loose
   values are brought back to T with fe_wcarry. */

FD_DEV void ge_p3_identity( ge_p3 & p ) { p.X = fe_zero(); p.Y = fe_one(); p.Z = fe_one(); p.T = fe_zero(); }

/* The completed -> projective/extended conversions share the 19x
   multiples of the operand used twice (T, and Y for p3). */
template<int FM = FD_CARRY_FOLD>
FD_DEV void ge_p1p1_to_p2( ge_p2 & r, ge_p1p1 const & p ) {
  fe19 t19; fe_x19( t19, p.T );
  fe_mul19<FM>( r.X, p.X, p.T, t19 ); fe_mul<FM>( r.Y, p.Y, p.Z ); fe_mul19<FM>( r.Z, p.Z, p.T, t19 );
}
template<int FM = FD_CARRY_FOLD>
FD_DEV void ge_p1p1_to_p3( ge_p3 & r, ge_p1p1 const & p ) {
  fe19 t19; fe_x19( t19, p.T );
  fe_mul19<FM>( r.X, p.X, p.T, t19 ); fe_mul19<FM>( r.Z, p.Z, p.T, t19 );
  fe19 y19; fe_x19( y19, p.Y );
  fe_mul19<FM>( r.Y, p.Z, p.Y, y19 ); fe_mul19<FM>( r.T, p.X, p.Y, y19 );
}

/* 2P for a=-1 twisted Edwards from (X:Y:Z) T -- eprint 2008/522 §4.4:
   4 squarings.  Out: X=E (T), Y=H (L), Z=G (L), T=F (T).  E = (X+Y)^2-H
   and F = 2Z^2-G are folded into their squarings' carry chains. */
template<int FM = FD_CARRY_FOLD>
FD_DEV void ge_dbl( ge_p1p1 & r, ge_p2 const & p ) {
  fe xx, yy, s;
  fe_sqr<FM>( xx, p.X );                  /* XX (T)               */
  fe_sqr<FM>( yy, p.Y );                  /* YY (T)               */
  fe_add( r.Y, yy, xx );              /* H = YY+XX (L)        */
  fe_sub( r.Z, yy, xx );              /* G = YY-XX (L)        */
  fe_add( s, p.X, p.Y );              /* X+Y (L)              */
  fe_sqr_sub<FM>( r.X, s, r.Y );          /* E = (X+Y)^2-H = 2XY  */
  fe_sqr2_sub<FM>( r.T, p.Z, r.Z );       /* F = 2ZZ-G            */
}

/* P + Q, P T, Q cached (already negated by the caller if needed)
   (eprint 2008/522 §4.2, 4 mul).  Out: X=E, Y=H, Z=G (L), T=F (T). */
template<int FM = FD_CARRY_FOLD>
FD_DEV void ge_add_cached( ge_p1p1 & r, ge_p3 const & p, ge_cached const & q ) {
  fe a, b, c, d;
  fe_add( a, p.Y, p.X );
  fe_sub( b, p.Y, p.X );
  fe_mul<FM>( a, a, q.YpX );              /* A (T) */
  fe_mul<FM>( b, b, q.YmX );              /* B (T) */
  fe_mul<FM>( c, q.T2d, p.T );            /* C (T) */
  fe_mul<FM>( d, p.Z, q.Z );
  fe_add( d, d, d );                  /* D = 2 Z1 Z2 (L) */
  fe_sub( r.X, a, b );                /* E (L) */
  fe_add( r.Y, a, b );                /* H (L) */
  fe_add( r.Z, d, c );                /* G (L) */
  fe_sub( r.T, d, c );                /* F */
  fe_wcarry( r.T, r.T );
}

/* P + Q, Q affine precomputed (Z=1), already negated if needed (3 mul). */
template<int FM = FD_CARRY_FOLD>
FD_DEV void ge_add_precomp( ge_p1p1 & r, ge_p3 const & p, ge_precomp const & q ) {
  fe a, b, c, d;
  fe_add( a, p.Y, p.X );
  fe_sub( b, p.Y, p.X );
  fe_mul<FM>( a, a, q.ypx );
  fe_mul<FM>( b, b, q.ymx );
  fe_mul<FM>( c, q.xy2d, p.T );
  fe_add( d, p.Z, p.Z );
  fe_sub( r.X, a, b );
  fe_add( r.Y, a, b );
  fe_add( r.Z, d, c );
  fe_sub( r.T, d, c );
  fe_wcarry( r.T, r.T );
}

/* -Q for a cached point: swap Y+X / Y-X, negate 2dT (T in -> L out) */
FD_DEV void ge_cached_cneg( ge_cached & q, int neg ) {
  fe t, n;
  fe_sel( t, neg, q.YmX, q.YpX );
  fe_sel( q.YmX, neg, q.YpX, q.YmX );
  q.YpX = t;
  fe_neg( n, q.T2d );
  fe_sel( q.T2d, neg, n, q.T2d );
}
FD_DEV void ge_precomp_cneg( ge_precomp & q, int neg ) {
  fe t, n;
  fe_sel( t, neg, q.ymx, q.ypx );
  fe_sel( q.ymx, neg, q.ypx, q.ymx );
  q.ypx = t;
  fe_neg( n, q.xy2d );
  fe_sel( q.xy2d, neg, n, q.xy2d );
}

/* p T */
template<int FM = FD_CARRY_FOLD>
FD_DEV void ge_p3_to_cached( ge_cached & r, ge_p3 const & p ) {
  fe_add( r.YpX, p.Y, p.X );
  fe_sub( r.YmX, p.Y, p.X );
  r.Z = p.Z;
  fe d2 = fe_d2();
  fe_mul<FM>( r.T2d, p.T, d2 );
}

template<int FM = FD_CARRY_FOLD>
FD_DEV void ge_p3_dbl( ge_p3 & r, ge_p3 const & p ) {
  ge_p2 q; q.X = p.X; q.Y = p.Y; q.Z = p.Z;
  ge_p1p1 t; ge_dbl<FM>( t, q ); ge_p1p1_to_p3<FM>( r, t );
}

template<int FM = FD_CARRY_FOLD>
FD_DEV void ge_p3_add( ge_p3 & r, ge_p3 const & p, ge_p3 const & q ) {
  ge_cached c; ge_p3_to_cached<FM>( c, q );
  ge_p1p1 t; ge_add_cached<FM>( t, p, c ); ge_p1p1_to_p3<FM>( r, t );
}

/* canonicalise in place (pack + unpack): any value with limbs < 2^31 -> T canonical */
FD_DEV void fe_canon( fe & a ) { u32 w[8]; fe_pack( w, a ); fe_unpack( a, w ); }

/* ---- decompression -------------------------------------------------- */

/* Decode 2 points at once (A and R), y from the 8 LE words with bit 255
   dropped.  Per point: x = (u v^3)(u v^7)^((p-5)/8), u = y^2-1,
   v = d y^2 + 1 (RFC 8032 5.1.3; fd_f25519_sqrt_ratio fd_f25519.c:105-143);
   v x^2 == u -> x, == -u -> x*sqrt(-1), else not a square.
   Returns per point: 0 ok, 1 not a square, 2 x==0 with sign bit set
   (the AVX-512 decode rejects this, avx512/fd_r43x6_ge.c:230-232; the
   portable decode negates 0 and accepts, fd_curve25519.c:41-43 -- the
   caller decides).  Outputs are canonical T with Z=1, T=xy. */
template<int FM = FD_CARRY_FOLD>
FD_DEV void fe_decode_uv( fe & u, fe & v, fe const & y ) {
  fe one = fe_one(), d = fe_d();
  fe_sqr<FM>( u, y );
  fe_mul<FM>( v, u, d );
  fe_sub( u, u, one );           /* u = y^2-1 (L) */
  fe_add( v, v, one );           /* v = dy^2+1 (L) */
}

template<int FM = FD_CARRY_FOLD>
FD_DEV void ge_decode1( ge_p3 & P, int & rc, u32 const w[ 8 ] ) {
  fe y; fe_unpack( y, w );
  int sgn = (int)(w[7] >> 31);
  fe u, v, t, x;
  fe_decode_uv<FM>( u, v, y );
  fe_sqr<FM>( t, v );
  fe_mul<FM>( t, t, v );             /* v^3 */
  fe_sqr<FM>( t, t );
  fe_mul<FM>( t, t, v );             /* v^7 */
  fe_mul<FM>( t, u, t );             /* u v^7 */
  fe_pow22523<FM>( x, t );
  /* u, v and u v^3 are recomputed rather than held across the 265-op
     chain: +5 field ops, -30 VGPRs */
  fe_decode_uv<FM>( u, v, y );
  fe_sqr<FM>( t, v );
  fe_mul<FM>( t, t, v );             /* v^3 */
  fe_mul<FM>( t, u, t );             /* u v^3 */
  fe_mul<FM>( x, x, t );
  fe_sqr<FM>( t, x );
  fe_mul<FM>( t, t, v );             /* v x^2 (T) */
  u32 wt[8], wu[8], wn[8];
  fe n; fe_add( n, t, u );       /* v x^2 + u */
  fe_pack( wt, t ); fe_pack( wu, u ); fe_pack( wn, n );
  u32 ne = 0, nz = 0;
#pragma unroll
  for( int k=0; k<8; k++ ) { ne |= wt[k] ^ wu[k]; nz |= wn[k]; }
  int ok = ne==0u, flip = nz==0u;
  fe i = fe_sqrtm1();
  fe_mul<FM>( t, x, i );
  fe_sel( x, !ok, t, x );
  u32 wx[8]; fe_pack( wx, x );
  u32 z = 0;
#pragma unroll
  for( int k=0; k<8; k++ ) z |= wx[k];
  fe_unpack( x, wx );            /* canonical */
  fe_neg( t, x ); fe_canon( t );
  fe_sel( x, (int)(wx[0] & 1u) != sgn, t, x );
  rc = ( ok | flip ) ? ( ( z==0u && sgn ) ? 2 : 0 ) : 1;
  P.X = x; P.Y = y; P.Z = fe_one(); fe_mul<FM>( P.T, x, y );
}

/* fd_ed25519_affine_is_small_order (fd_curve25519.h:88-118): on a decoded
   (Z=1) point, X==0 | Y==0 | Y==y0 | Y==y1. */
FD_DEV int ge_affine_is_small_order( ge_p3 const & p ) {
  u32 const y0[8] = FD_Y0_W, y1[8] = FD_Y1_W;
  u32 wy[8]; fe_pack( wy, p.Y );
  u32 zx = 0, zy = 0, e0 = 0, e1 = 0;
  u32 wx[8]; fe_pack( wx, p.X );
#pragma unroll
  for( int k=0; k<8; k++ ) { zx |= wx[k]; zy |= wy[k]; e0 |= wy[k] ^ y0[k]; e1 |= wy[k] ^ y1[k]; }
  return (zx==0u) | (zy==0u) | (e0==0u) | (e1==0u);
}

/* ---- scalars mod l ---------------------------------------------------- */

/* S < l, S as 8 LE words (fd_curve25519_scalar_validate: S <= l-1). */
FD_DEV int sc_is_canonical( u32 const s[ 8 ] ) {
  u32 const lw[8] = { 0x5cf5d3edu, 0x5812631au, 0xa2f79cd6u, 0x14def9deu, 0u, 0u, 0u, 0x10000000u };
  int lt = 0, decided = 0;
#pragma unroll
  for( int i=7; i>=0; i-- ) {
    int l = s[i] < lw[i], g = s[i] > lw[i];
    lt = decided ? lt : l;
    decided |= (l | g);
  }
  return decided ? lt : 0; /* equal to l -> not canonical */
}

/* bits [bit, bit+nbits) of the 512-bit input (nbits <= 29, compile-time bit): one funnel
   shift of two words (a 64-bit combine of the pair made the compiler spill the input to
   scratch and reload it with unaligned 64-bit loads) */
FD_DEV i64 sc_get21( u32 const w[ 16 ], int bit, int nbits ) {
  int wi = bit >> 5, sh = bit & 31;
  u32 hi = wi+1 < 16 ? w[wi+1] : 0u;
  u32 x = __builtin_amdgcn_alignbit( hi, w[wi], (u32)sh );
  return (i64)( x & ((1u << nbits) - 1u) );
}

FD_DEV void sc_fold( i64 * t, int j ) {
  i64 v = t[j];
  t[j-12] += v * 666643; t[j-11] += v * 470296; t[j-10] += v * 654183;
  t[j- 9] -= v * 997805; t[j- 8] += v * 136657; t[j- 7] -= v * 683901;
  t[j] = 0;
}
FD_DEV void sc_carry_round( i64 * t, int i ) { i64 c = (t[i] + (1L<<20)) >> 21; t[i+1] += c; t[i] -= c * (1L<<21); }
FD_DEV void sc_carry_floor( i64 * t, int i ) { i64 c = t[i] >> 21; t[i+1] += c; t[i] -= c * (1L<<21); }

/* 512-bit (16 LE words) -> mod l (8 LE words).  Signed 21-bit limbs,
   2^252 = -c (mod l); same folding schedule as
   fd_curve25519_scalar_reduce (fd_curve25519_scalar.c:3-110). */
FD_DEV void sc_reduce( u32 out[ 8 ], u32 const in[ 16 ] ) {
  i64 t[25];
#pragma unroll
  for( int i=0; i<23; i++ ) t[i] = sc_get21( in, 21*i, 21 );
  t[23] = sc_get21( in, 483, 29 ); t[24] = 0;
#pragma unroll
  for( int j=23; j>=18; j-- ) sc_fold( t, j );
#pragma unroll
  for( int i=6; i<=16; i+=2 ) sc_carry_round( t, i );
#pragma unroll
  for( int i=7; i<=15; i+=2 ) sc_carry_round( t, i );
#pragma unroll
  for( int j=17; j>=12; j-- ) sc_fold( t, j );
#pragma unroll
  for( int i=0; i<=10; i+=2 ) sc_carry_round( t, i );
#pragma unroll
  for( int i=1; i<=11; i+=2 ) sc_carry_round( t, i );
  sc_fold( t, 12 );
#pragma unroll
  for( int i=0; i<=11; i++ ) sc_carry_floor( t, i );
  sc_fold( t, 12 );
#pragma unroll
  for( int i=0; i<=10; i++ ) sc_carry_floor( t, i );
  /* pack 12 x 21-bit limbs (t[11] may hold bit 252) */
  u64 acc = 0; int accb = 0, o = 0;
#pragma unroll
  for( int i=0; i<12; i++ ) {
    acc |= (u64)t[i] << accb; accb += 21;
    if( accb >= 32 ) { out[o++] = (u32)acc; acc >>= 32; accb -= 32; }
  }
  while( o < 8 ) { out[o++] = (u32)acc; acc >>= 32; }
}
