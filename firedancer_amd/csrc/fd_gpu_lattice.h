#pragma once
/* fd_gpu_lattice.h -- half-size scalars for the verification equation
   (device code; the same source also compiles as host C for the tests,
   tests/test_lattice.py through fd_lat_host.c).

   The reference checks R == [S]B - [k]A as points (fd_ed25519_verify,
   src/ballet/ed25519/fd_ed25519_user.c:204-226: fd_ed25519_double_scalar_
   mul_base, then fd_ed25519_point_eq_z1), i.e. D = [S]B - [k]A - R == O,
   with k < l a 253-bit hash.  The reduction of Pornin (eprint 2020/454,
   "Optimized lattice basis reduction in dimension 2, and fast Schnorr and
   EdDSA signature verification") rewrites that check with two ~128-bit
   scalars, so the double-and-add walk needs 128 doublings instead of 252:

     find c0, c1 with c0 == c1 k (mod 8 l), c1 odd, |c0|, |c1| ~ 2^128
     Q = [c1 S mod l]B + [c0](-A) + [c1](-R)

   Then Q = [c1] D exactly:
     [c1 S mod l]B = [c1 S]B            (B has order l)
     [c0]A         = [c1 k]A            (every curve point has order | 8 l)
   and [c1] is a bijection of the curve group (order 8 l, gcd(c1, 8 l) = 1
   because c1 is odd and 0 < |c1| < l), so Q == O  <=>  D == O: the same
   verdict as the reference for every input, including A and R with a
   torsion component.  (Modulus l alone would leave [c1 k - c0]A = a torsion
   point; an even c1 would map a torsion D to O.)

   (c0, c1) is a short vector of the lattice {(x, y): x == y k mod 8l},
   basis (8l, 0), (k, 1): a Lehmer-style Euclid on (8l, k) stopped where
   the remainder drops under 2^128 (remainder r, cofactor t: r == t k,
   |t| <= 8l / r_prev < 2^127).  Every step is an integer row operation on
   the two lattice vectors, so c0 == c1 k (mod 8l) holds whatever the
   approximations decide; the caller re-checks the congruence anyway
   (mod 8 and, with sc_reduce, mod l).  For random k the pair fits 131
   bits in 99.8 % of cases and ~140 in the rest (no short vector with c1
   odd); the walk's length follows the largest scalar of each wave.  A
   signature whose reduction fails a bound (not seen for hash-distributed
   k; k = l - 1 is one) takes the full 253-bit walk.

   Each outer iteration takes the top 64 bits of both remainders and runs
   binary Euclid steps on them (a -= b << s), accumulating the 2x2
   cofactor matrix (entries < 2^31), then applies the matrix once to the
   256-bit remainders and the 160-bit cofactors: 5 outer iterations of
   ~22 cheap 64-bit steps each. */

#include <stdint.h>

#ifndef FD_LAT_FN
#if defined(__HIPCC__)
#define FD_LAT_FN __device__ __forceinline__
#else
#define FD_LAT_FN static inline
#endif
#endif

#define FD_LAT_MAXIT  10      /* outer iterations (5 for all but rare k) */
#define FD_LAT_MAXIN  64      /* 64-bit steps per outer iteration */
#define FD_LAT_BITS   159     /* |c0|, |c1| < 2^159 (40 signed radix-16 digits); typically < 2^131 */

/* 8 l, little-endian words */
#define FD_LAT_N8L { 0xe7ae9f68u, 0xc09318d2u, 0x17bce6b2u, 0xa6f7cef5u, 0u, 0u, 0u, 0x80000000u }

/* bit length of an 8-word value */
FD_LAT_FN int fd_lat_bitlen8( uint32_t const x[ 8 ] ) {
  int b = 0;
#pragma unroll
  for( int i=0; i<8; i++ ) b = x[i] ? 32*i + 32 - __builtin_clz( x[i] ) : b;
  return b;
}

FD_LAT_FN int fd_lat_clz64( uint64_t x ) { return __builtin_clzll( x ); }   /* x != 0 */

/* x[w] (0 for w >= 8) without a lane-variable array index (no scratch) */
FD_LAT_FN uint32_t fd_lat_word( uint32_t const x[ 8 ], int w ) {
  uint32_t r = 0u;
#pragma unroll
  for( int i=0; i<8; i++ ) r = ( w==i ) ? x[i] : r;
  return r;
}

/* bits [sh, sh+64) of an 8-word value */
FD_LAT_FN uint64_t fd_lat_bits64( uint32_t const x[ 8 ], int sh ) {
  int w = sh >> 5, r = sh & 31;
  uint64_t x0 = fd_lat_word( x, w ), x1 = fd_lat_word( x, w+1 ), x2 = fd_lat_word( x, w+2 );
  uint64_t lo = ( ( x1 << 32 ) | x0 ) >> r;
  uint64_t hi = ( ( x2 << 32 ) | x1 ) >> r;
  return ( hi << 32 ) | ( lo & 0xffffffffUL );
}

/* d = x P - y Q (x, y < 2^31): |d| -> out (8 words), returns 1 if d < 0;
   *ovf set if |d| >= 2^256 */
FD_LAT_FN int fd_lat_comb8( uint32_t out[ 8 ], uint32_t x, uint32_t const P[ 8 ], uint32_t y, uint32_t const Q[ 8 ],
                            int * ovf ) {
  uint64_t cp = 0, cq = 0; int64_t br = 0;
  uint32_t d[ 8 ];
#pragma unroll
  for( int i=0; i<8; i++ ) {
    uint64_t p = (uint64_t)x * P[i] + cp; cp = p >> 32;
    uint64_t q = (uint64_t)y * Q[i] + cq; cq = q >> 32;
    int64_t t = (int64_t)( p & 0xffffffffUL ) - (int64_t)( q & 0xffffffffUL ) + br;
    d[i] = (uint32_t)t; br = t >> 32;
  }
  int64_t top = (int64_t)cp - (int64_t)cq + br;
  int neg = top < 0;
  uint32_t m = neg ? 0xffffffffu : 0u;
  uint64_t c = (uint64_t)neg;
#pragma unroll
  for( int i=0; i<8; i++ ) { uint64_t v = (uint64_t)( d[i] ^ m ) + c; out[i] = (uint32_t)v; c = v >> 32; }
  uint32_t tw = ( (uint32_t)top ^ m ) + (uint32_t)c;
  *ovf |= tw != 0u;
  return neg;
}

/* out = +-(x P - y Q) mod 2^160 on two's-complement 5-word values (minus if neg) */
FD_LAT_FN void fd_lat_combT( uint32_t out[ 5 ], uint32_t x, uint32_t const P[ 5 ], uint32_t y, uint32_t const Q[ 5 ],
                             int neg ) {
  uint64_t cp = 0, cq = 0; int64_t br = 0;
  uint32_t d[ 5 ];
#pragma unroll
  for( int i=0; i<5; i++ ) {
    uint64_t p = (uint64_t)x * P[i] + cp; cp = p >> 32;
    uint64_t q = (uint64_t)y * Q[i] + cq; cq = q >> 32;
    int64_t t = (int64_t)( p & 0xffffffffUL ) - (int64_t)( q & 0xffffffffUL ) + br;
    d[i] = (uint32_t)t; br = t >> 32;
  }
  uint32_t m = neg ? 0xffffffffu : 0u;
  uint64_t c = (uint64_t)( neg != 0 );
#pragma unroll
  for( int i=0; i<5; i++ ) { uint64_t v = (uint64_t)( d[i] ^ m ) + c; out[i] = (uint32_t)v; c = v >> 32; }
}

FD_LAT_FN int fd_lat_lt8( uint32_t const a[ 8 ], uint32_t const b[ 8 ] ) {   /* a < b */
  int lt = 0, dec = 0;
#pragma unroll
  for( int i=7; i>=0; i-- ) { int l = a[i] < b[i], g = a[i] > b[i]; lt = dec ? lt : l; dec |= l | g; }
  return lt;
}

/* |t| of a two's-complement 5-word value; returns the sign */
FD_LAT_FN int fd_lat_abs5( uint32_t out[ 5 ], uint32_t const t[ 5 ] ) {
  int neg = (int)( t[4] >> 31 );
  uint32_t m = neg ? 0xffffffffu : 0u;
  uint64_t c = (uint64_t)neg;
#pragma unroll
  for( int i=0; i<5; i++ ) { uint64_t v = (uint64_t)( t[i] ^ m ) + c; out[i] = (uint32_t)v; c = v >> 32; }
  return neg;
}

FD_LAT_FN double fd_lat_dbl( uint32_t const x[], int nw ) {
  double f = 0.0;
  for( int i=nw-1; i>=0; i-- ) f = f * 4294967296.0 + (double)x[i];
  return f;
}

/* k (8 LE words, k < l) -> c0 >= 0 (5 words), |c1| (5 words, odd), sign of c1,
   with c0 == c1 k (mod 8l) by construction and both below 2^FD_LAT_BITS.
   Returns 0 when a bound fails (the caller takes the full-length walk). */
FD_LAT_FN int fd_lat_halfsize( uint32_t c0[ 5 ], uint32_t c1m[ 5 ], int * c1neg, uint32_t const k[ 8 ] ) {
  uint32_t R0[ 8 ] = FD_LAT_N8L, R1[ 8 ], T0[ 5 ] = { 0u, 0u, 0u, 0u, 0u }, T1[ 5 ] = { 1u, 0u, 0u, 0u, 0u };
#pragma unroll
  for( int i=0; i<8; i++ ) R1[i] = k[i];
  int ovf = 0;
#pragma unroll 1
  for( int it=0; it<FD_LAT_MAXIT; it++ ) {
    if( !( R1[4] | R1[5] | R1[6] | R1[7] ) ) break;       /* remainder under 2^128 */
    int L = fd_lat_bitlen8( R0 );                          /* R0 >= R1 >= 2^128: L >= 129 */
    int sh = L - 64;
    uint64_t a = fd_lat_bits64( R0, sh ), b = fd_lat_bits64( R1, sh );
    int stopb = 192 - L;                                   /* b < 2^stopb: R1 would drop under ~2^128 */
    uint64_t thr = stopb > 33 ? ( 1UL << stopb ) : ( 1UL << 33 );
    uint32_t m00 = 1u, m01 = 0u, m10 = 0u, m11 = 1u;
    int steps = 0;
#pragma unroll 1
    for( int j=0; j<FD_LAT_MAXIN; j++ ) {
      if( b < thr ) break;
      int s = fd_lat_clz64( b ) - fd_lat_clz64( a );
      if( s >= 31 ) break;
      uint64_t bs = b << s;
      if( bs > a ) { s--; bs >>= 1; }
      uint64_t n00 = (uint64_t)m00 + ( (uint64_t)m10 << s ), n01 = (uint64_t)m01 + ( (uint64_t)m11 << s );
      if( ( n00 | n01 ) >> 31 ) break;
      a -= bs; m00 = (uint32_t)n00; m01 = (uint32_t)n01; steps++;
      if( a < b ) {
        uint64_t ta = a; a = b; b = ta;
        uint32_t t0 = m00; m00 = m10; m10 = t0;
        uint32_t t1 = m01; m01 = m11; m11 = t1;
      }
    }
    if( !steps ) {                                         /* R0 >> R1: R0 -= 2^s R1, s <= 30 */
      int s = L - fd_lat_bitlen8( R1 ) - 1;
      s = s < 0 ? 0 : ( s > 30 ? 30 : s );
      m00 = 1u; m01 = 1u << s; m10 = 0u; m11 = 1u;
    }
    /* row k of the matrix applied to both lattice vectors, then |.| */
    uint32_t nR0[ 8 ], nR1[ 8 ], nT0[ 5 ], nT1[ 5 ];
    int n0 = fd_lat_comb8( nR0, m00, R0, m01, R1, &ovf );
    int n1 = fd_lat_comb8( nR1, m11, R1, m10, R0, &ovf );
    fd_lat_combT( nT0, m00, T0, m01, T1, n0 );
    fd_lat_combT( nT1, m11, T1, m10, T0, n1 );
    int sw = fd_lat_lt8( nR0, nR1 );
#pragma unroll
    for( int i=0; i<8; i++ ) { R0[i] = sw ? nR1[i] : nR0[i]; R1[i] = sw ? nR0[i] : nR1[i]; }
#pragma unroll
    for( int i=0; i<5; i++ ) { T0[i] = sw ? nT1[i] : nT0[i]; T1[i] = sw ? nT0[i] : nT1[i]; }
  }
  if( ovf | R1[4] | R1[5] | R1[6] | R1[7] ) return 0;

  uint32_t cr[ 8 ], ct[ 5 ];
  if( T1[0] & 1u ) {                                       /* (R1, T1): c1 odd */
#pragma unroll
    for( int i=0; i<8; i++ ) cr[i] = R1[i];
#pragma unroll
    for( int i=0; i<5; i++ ) ct[i] = T1[i];
  } else {
    /* T1 even -> T0 odd (the cofactor column has gcd 1): the shortest
       (R0 - j R1, T0 - j T1), j ~ (R0 - |T0|) / (R1 + |T1|), j or j+1 */
    uint32_t a0[ 5 ], a1[ 5 ];
    fd_lat_abs5( a0, T0 ); fd_lat_abs5( a1, T1 );
    double q = ( fd_lat_dbl( R0, 8 ) - fd_lat_dbl( a0, 5 ) ) / ( fd_lat_dbl( R1, 8 ) + fd_lat_dbl( a1, 5 ) );
    if( !( q < 2147483647.0 ) ) return 0;                  /* also NaN */
    uint32_t j = q > 0.0 ? (uint32_t)q : 0u;
    int best = 1 << 20;
#pragma unroll 1
    for( uint32_t jj=j; jj<=j+1u; jj++ ) {
      uint32_t dr[ 8 ], dt[ 5 ], da[ 5 ];
      int o2 = 0;
      int ng = fd_lat_comb8( dr, 1u, R0, jj, R1, &o2 );
      fd_lat_combT( dt, 1u, T0, jj, T1, ng );
      fd_lat_abs5( da, dt );
      uint32_t h = dr[5] | dr[6] | dr[7];
      int bits = ( o2 | ( h != 0u ) ) ? ( 1 << 19 ) : fd_lat_bitlen8( dr );
      uint32_t da8[ 8 ] = { da[0], da[1], da[2], da[3], da[4], 0u, 0u, 0u };
      int bt = fd_lat_bitlen8( da8 );
      bits = bits > bt ? bits : bt;
      if( bits < best ) {
        best = bits;
#pragma unroll
        for( int i=0; i<8; i++ ) cr[i] = dr[i];
#pragma unroll
        for( int i=0; i<5; i++ ) ct[i] = dt[i];
      }
    }
  }
  if( cr[5] | cr[6] | cr[7] ) return 0;
  *c1neg = fd_lat_abs5( c1m, ct );
#pragma unroll
  for( int i=0; i<5; i++ ) c0[i] = cr[i];
  /* bounds: both < 2^FD_LAT_BITS (word 4 holds bits 128..159), |c1| odd */
  uint32_t lim = 1u << ( FD_LAT_BITS - 128 );
  return ( c0[4] < lim ) & ( c1m[4] < lim ) & (int)( c1m[0] & 1u );
}
