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
struct ge_p1p1  { fe X, Y, Z, T; };     /* completed: (X:Z),(Y:T)        */
struct ge_cached{ fe YpX, YmX, Z, T2d; };
struct ge_precomp{ fe ypx, ymx, xy2d; };/* affine, Z = 1                 */

FD_DEV void ge_p3_identity( ge_p3 & p ) { p.X = fe_zero(); p.Y = fe_one(); p.Z = fe_one(); p.T = fe_zero(); }

FD_DEV void ge_p1p1_to_p2( ge_p2 & r, ge_p1p1 const & p ) {
  fe_mul( r.X, p.X, p.T ); fe_mul( r.Y, p.Y, p.Z ); fe_mul( r.Z, p.Z, p.T );
}
FD_DEV void ge_p1p1_to_p3( ge_p3 & r, ge_p1p1 const & p ) {
  fe_mul( r.X, p.X, p.T ); fe_mul( r.Y, p.Y, p.Z ); fe_mul( r.Z, p.Z, p.T ); fe_mul( r.T, p.X, p.Y );
}

/* 2P for a=-1 twisted Edwards from (X:Y:Z) -- eprint 2008/522 §4.4:
   4 squarings. */
FD_DEV void ge_dbl( ge_p1p1 & r, ge_p2 const & p ) {
  fe t0;
  fe_sqr( r.X, p.X );                 /* XX        */
  fe_sqr( r.Z, p.Y );                 /* YY        */
  fe_sqr( r.T, p.Z );                 /* ZZ        */
  fe_add( r.T, r.T, r.T );            /* 2ZZ       */
  fe_add( r.Y, p.X, p.Y );
  fe_sqr( t0, r.Y );                  /* (X+Y)^2   */
  fe_add( r.Y, r.Z, r.X );            /* YY+XX     */
  fe_sub( r.Z, r.Z, r.X );            /* YY-XX     */
  fe_sub( r.X, t0, r.Y );             /* 2XY       */
  fe_sub( r.T, r.T, r.Z );            /* 2ZZ-YY+XX */
}

/* P + (neg ? -Q : Q), Q cached (eprint 2008/522 §4.2, 4 mul).  -Q swaps
   YpX/YmX and negates T2d, i.e. swaps the roles of D+C and D-C. */
FD_DEV void ge_add_cached( ge_p1p1 & r, ge_p3 const & p, ge_cached const & q, int neg ) {
  fe a, b, c, d, qp, qm;
  fe_sel( qp, neg, q.YmX, q.YpX );
  fe_sel( qm, neg, q.YpX, q.YmX );
  fe_add( a, p.Y, p.X );
  fe_sub( b, p.Y, p.X );
  fe_mul( a, a, qp );
  fe_mul( b, b, qm );
  fe_mul( c, q.T2d, p.T );
  fe_mul( d, p.Z, q.Z );
  fe_add( d, d, d );
  fe_sub( r.X, a, b );
  fe_add( r.Y, a, b );
  fe_add( a, d, c );
  fe_sub( b, d, c );
  fe_sel( r.Z, neg, b, a );
  fe_sel( r.T, neg, a, b );
}

/* P + (neg ? -Q : Q), Q affine precomputed (3 mul). */
FD_DEV void ge_add_precomp( ge_p1p1 & r, ge_p3 const & p, ge_precomp const & q, int neg ) {
  fe a, b, c, d, qp, qm;
  fe_sel( qp, neg, q.ymx, q.ypx );
  fe_sel( qm, neg, q.ypx, q.ymx );
  fe_add( a, p.Y, p.X );
  fe_sub( b, p.Y, p.X );
  fe_mul( a, a, qp );
  fe_mul( b, b, qm );
  fe_mul( c, q.xy2d, p.T );
  fe_add( d, p.Z, p.Z );
  fe_sub( r.X, a, b );
  fe_add( r.Y, a, b );
  fe_add( a, d, c );
  fe_sub( b, d, c );
  fe_sel( r.Z, neg, b, a );
  fe_sel( r.T, neg, a, b );
}

FD_DEV void ge_p3_to_cached( ge_cached & r, ge_p3 const & p ) {
  fe_add( r.YpX, p.Y, p.X );
  fe_sub( r.YmX, p.Y, p.X );
  r.Z = p.Z;
  fe d2 = fe_d2();
  fe_mul( r.T2d, p.T, d2 );
}

FD_DEV void ge_p3_dbl( ge_p3 & r, ge_p3 const & p ) {
  ge_p2 q; q.X = p.X; q.Y = p.Y; q.Z = p.Z;
  ge_p1p1 t; ge_dbl( t, q ); ge_p1p1_to_p3( r, t );
}

FD_DEV void ge_p3_add( ge_p3 & r, ge_p3 const & p, ge_p3 const & q ) {
  ge_cached c; ge_p3_to_cached( c, q );
  ge_p1p1 t; ge_add_cached( t, p, c, 0 ); ge_p1p1_to_p3( r, t );
}

/* ---- decompression -------------------------------------------------- */

/* Decode 2 points at once (A and R), y from the 8 LE words with bit 255
   dropped.  Per point: x = (u v^3)(u v^7)^((p-5)/8), u = y^2-1,
   v = d y^2 + 1 (RFC 8032 5.1.3; fd_f25519_sqrt_ratio fd_f25519.c:105-143);
   v x^2 == u -> x, == -u -> x*sqrt(-1), else not a square.
   Returns per point: 0 ok, 1 not a square, 2 x==0 with sign bit set
   (the AVX-512 decode rejects this, avx512/fd_r43x6_ge.c:230-232; the
   portable decode negates 0 and accepts, fd_curve25519.c:41-43 -- the
   caller decides).  On 0 or 2, x has the requested sign. */
FD_DEV void ge_decode2( ge_p3 & Pa, int & ra, u32 const wa[ 8 ],
                        ge_p3 & Pb, int & rb, u32 const wb[ 8 ] ) {
  fe one = fe_one(), d = fe_d();
  fe ya, yb; fe_from_words( ya, wa ); fe_from_words( yb, wb );
  int sa = (int)(wa[7] >> 31), sb = (int)(wb[7] >> 31);
  fe ua, ub, va, vb, t, s;
  fe_sqr( ua, ya );              fe_sqr( ub, yb );
  fe_mul( va, ua, d );           fe_mul( vb, ub, d );
  fe_sub( ua, ua, one );         fe_sub( ub, ub, one );
  fe_add( va, va, one );         fe_add( vb, vb, one );
  fe v3a, v3b, uv3a, uv3b, uv7a, uv7b;
  fe_sqr( t, va );               fe_sqr( s, vb );
  fe_mul( v3a, t, va );          fe_mul( v3b, s, vb );
  fe_mul( uv3a, ua, v3a );       fe_mul( uv3b, ub, v3b );
  fe_sqr( t, v3a );              fe_sqr( s, v3b );
  fe_mul( t, t, va );            fe_mul( s, s, vb );          /* v^7 */
  fe_mul( uv7a, ua, t );         fe_mul( uv7b, ub, s );
  fe xa, xb;
  fe_pow22523_2( xa, uv7a, xb, uv7b );
  fe_mul( xa, xa, uv3a );        fe_mul( xb, xb, uv3b );
  /* check */
  fe_sqr( t, xa );               fe_sqr( s, xb );
  fe_mul( t, t, va );            fe_mul( s, s, vb );          /* v x^2 */
  fe na, nb;
  fe_sub( na, t, ua );           fe_sub( nb, s, ub );
  int oka = fe_is_zero( na ),    okb = fe_is_zero( nb );
  fe_add( na, t, ua );           fe_add( nb, s, ub );
  int fla = fe_is_zero( na ),    flb = fe_is_zero( nb );
  fe i = fe_sqrtm1();
  fe_mul( t, xa, i );            fe_mul( s, xb, i );
  fe_sel( xa, !oka, t, xa );     fe_sel( xb, !okb, s, xb );
  /* sign */
  fe_canon( xa, xa );            fe_canon( xb, xb );
  u32 za = 0, zb = 0;
#pragma unroll
  for( int k=0; k<8; k++ ) { za |= xa.v[k]; zb |= xb.v[k]; }
  fe_neg( t, xa );               fe_neg( s, xb );
  fe_sel( xa, (int)(xa.v[0] & 1u) != sa, t, xa );
  fe_sel( xb, (int)(xb.v[0] & 1u) != sb, s, xb );
  ra = ( oka | fla ) ? ( ( za==0u && sa ) ? 2 : 0 ) : 1;
  rb = ( okb | flb ) ? ( ( zb==0u && sb ) ? 2 : 0 ) : 1;
  Pa.X = xa; Pa.Y = ya; Pa.Z = one; fe_mul( Pa.T, xa, ya );
  Pb.X = xb; Pb.Y = yb; Pb.Z = one; fe_mul( Pb.T, xb, yb );
}

/* fd_ed25519_affine_is_small_order (fd_curve25519.h:88-118): on a decoded
   (Z=1) point, X==0 | Y==0 | Y==y0 | Y==y1. */
FD_DEV int ge_affine_is_small_order( ge_p3 const & p ) {
  fe y0 = fe_y0(), y1 = fe_y1();
  return fe_is_zero( p.X ) | fe_is_zero( p.Y ) | fe_eq( p.Y, y0 ) | fe_eq( p.Y, y1 );
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

FD_DEV i64 sc_get21( u32 const w[ 16 ], int bit, int nbits ) {
  int wi = bit >> 5, sh = bit & 31;
  u64 x = (u64)w[wi] | ( wi+1 < 16 ? ((u64)w[wi+1] << 32) : 0UL );
  return (i64)( (x >> sh) & ((1UL << nbits) - 1UL) );
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
