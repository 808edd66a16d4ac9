/* fd_ed25519_oracle.c -- TEST INFRASTRUCTURE ONLY (see header).

   A from-scratch, portable C restatement of the reference's ed25519
   verify path, written to be obviously correct rather than fast:
   GF(2^255-19) in radix 2^51 (5 x u64 limbs, unsigned __int128
   products), extended twisted Edwards points, wNAF double-scalar
   multiplication.  Each function cites the reference code it restates.

   Result-code semantics follow the reference AVX-512 build by default
   (FDGPU_SEMANTICS_AVX512) or the portable build (FDGPU_SEMANTICS_REF);
   SURVEY.md §0.2 / §8a-a3. */

#include "fd_ed25519_oracle.h"

#include <string.h>
#include <pthread.h>

typedef unsigned __int128 u128;

/* ===================================================================
   SHA-512 (FIPS 180-4).  Restates src/ballet/sha512/fd_sha512.c:265-398
   (init/append/fini) and the block function fd_sha512_core_ref
   (fd_sha512.c:128-230).
   =================================================================== */

static uint64_t const sha512_k[ 80 ] = {
  0x428a2f98d728ae22UL, 0x7137449123ef65cdUL, 0xb5c0fbcfec4d3b2fUL, 0xe9b5dba58189dbbcUL,
  0x3956c25bf348b538UL, 0x59f111f1b605d019UL, 0x923f82a4af194f9bUL, 0xab1c5ed5da6d8118UL,
  0xd807aa98a3030242UL, 0x12835b0145706fbeUL, 0x243185be4ee4b28cUL, 0x550c7dc3d5ffb4e2UL,
  0x72be5d74f27b896fUL, 0x80deb1fe3b1696b1UL, 0x9bdc06a725c71235UL, 0xc19bf174cf692694UL,
  0xe49b69c19ef14ad2UL, 0xefbe4786384f25e3UL, 0x0fc19dc68b8cd5b5UL, 0x240ca1cc77ac9c65UL,
  0x2de92c6f592b0275UL, 0x4a7484aa6ea6e483UL, 0x5cb0a9dcbd41fbd4UL, 0x76f988da831153b5UL,
  0x983e5152ee66dfabUL, 0xa831c66d2db43210UL, 0xb00327c898fb213fUL, 0xbf597fc7beef0ee4UL,
  0xc6e00bf33da88fc2UL, 0xd5a79147930aa725UL, 0x06ca6351e003826fUL, 0x142929670a0e6e70UL,
  0x27b70a8546d22ffcUL, 0x2e1b21385c26c926UL, 0x4d2c6dfc5ac42aedUL, 0x53380d139d95b3dfUL,
  0x650a73548baf63deUL, 0x766a0abb3c77b2a8UL, 0x81c2c92e47edaee6UL, 0x92722c851482353bUL,
  0xa2bfe8a14cf10364UL, 0xa81a664bbc423001UL, 0xc24b8b70d0f89791UL, 0xc76c51a30654be30UL,
  0xd192e819d6ef5218UL, 0xd69906245565a910UL, 0xf40e35855771202aUL, 0x106aa07032bbd1b8UL,
  0x19a4c116b8d2d0c8UL, 0x1e376c085141ab53UL, 0x2748774cdf8eeb99UL, 0x34b0bcb5e19b48a8UL,
  0x391c0cb3c5c95a63UL, 0x4ed8aa4ae3418acbUL, 0x5b9cca4f7763e373UL, 0x682e6ff3d6b2b8a3UL,
  0x748f82ee5defb2fcUL, 0x78a5636f43172f60UL, 0x84c87814a1f0ab72UL, 0x8cc702081a6439ecUL,
  0x90befffa23631e28UL, 0xa4506cebde82bde9UL, 0xbef9a3f7b2c67915UL, 0xc67178f2e372532bUL,
  0xca273eceea26619cUL, 0xd186b8c721c0c207UL, 0xeada7dd6cde0eb1eUL, 0xf57d4f7fee6ed178UL,
  0x06f067aa72176fbaUL, 0x0a637dc5a2c898a6UL, 0x113f9804bef90daeUL, 0x1b710b35131c471bUL,
  0x28db77f523047d84UL, 0x32caab7b40c72493UL, 0x3c9ebe0a15c9bebcUL, 0x431d67c49c100d4cUL,
  0x4cc5d4becb3e42b6UL, 0x597f299cfc657e2aUL, 0x5fcb6fab3ad6faecUL, 0x6c44198c4a475817UL
};

static inline uint64_t rotr64( uint64_t x, int n ) { return (x>>n) | (x<<(64-n)); }

static inline uint64_t load_be64( uint8_t const * p ) {
  uint64_t r = 0; for( int i=0; i<8; i++ ) r = (r<<8) | p[i]; return r;
}

static void
sha512_block( uint64_t h[ 8 ], uint8_t const blk[ 128 ] ) {
  uint64_t w[ 80 ];
  for( int t=0; t<16; t++ ) w[t] = load_be64( blk + 8*t );
  for( int t=16; t<80; t++ ) {
    uint64_t s0 = rotr64( w[t-15], 1 ) ^ rotr64( w[t-15], 8 ) ^ (w[t-15]>>7);
    uint64_t s1 = rotr64( w[t- 2],19 ) ^ rotr64( w[t- 2],61 ) ^ (w[t- 2]>>6);
    w[t] = w[t-16] + s0 + w[t-7] + s1;
  }
  uint64_t a=h[0], b=h[1], c=h[2], d=h[3], e=h[4], f=h[5], g=h[6], hh=h[7];
  for( int t=0; t<80; t++ ) {
    uint64_t S1 = rotr64( e,14 ) ^ rotr64( e,18 ) ^ rotr64( e,41 );
    uint64_t ch = (e & f) ^ (~e & g);
    uint64_t t1 = hh + S1 + ch + sha512_k[t] + w[t];
    uint64_t S0 = rotr64( a,28 ) ^ rotr64( a,34 ) ^ rotr64( a,39 );
    uint64_t mj = (a & b) ^ (a & c) ^ (b & c);
    uint64_t t2 = S0 + mj;
    hh = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
  }
  h[0]+=a; h[1]+=b; h[2]+=c; h[3]+=d; h[4]+=e; h[5]+=f; h[6]+=g; h[7]+=hh;
}

typedef struct { uint64_t h[8]; uint8_t buf[128]; size_t buf_used; uint64_t bit_cnt; } sha512_t;

static void sha512_init( sha512_t * s ) {
  static uint64_t const iv[8] = {
    0x6a09e667f3bcc908UL, 0xbb67ae8584caa73bUL, 0x3c6ef372fe94f82bUL, 0xa54ff53a5f1d36f1UL,
    0x510e527fade682d1UL, 0x9b05688c2b3e6c1fUL, 0x1f83d9abfb41bd6bUL, 0x5be0cd19137e2179UL };
  memcpy( s->h, iv, sizeof(iv) ); s->buf_used = 0; s->bit_cnt = 0;
}

static void sha512_append( sha512_t * s, uint8_t const * p, size_t sz ) {
  s->bit_cnt += (uint64_t)sz << 3;
  while( sz ) {
    size_t n = 128 - s->buf_used; if( n > sz ) n = sz;
    memcpy( s->buf + s->buf_used, p, n );
    s->buf_used += n; p += n; sz -= n;
    if( s->buf_used==128 ) { sha512_block( s->h, s->buf ); s->buf_used = 0; }
  }
}

static void sha512_fini( sha512_t * s, uint8_t out[ 64 ] ) {
  uint64_t bits = s->bit_cnt;
  uint8_t pad = 0x80;
  sha512_append( s, &pad, 1 );
  uint8_t z = 0;
  while( s->buf_used != 112 ) sha512_append( s, &z, 1 );
  uint8_t len[16] = {0};
  for( int i=0; i<8; i++ ) len[15-i] = (uint8_t)(bits >> (8*i));
  sha512_append( s, len, 16 );
  for( int i=0; i<8; i++ ) for( int j=0; j<8; j++ ) out[8*i+j] = (uint8_t)(s->h[i] >> (56-8*j));
}

void oracle_sha512( uint8_t const * in, size_t sz, uint8_t out[ 64 ] ) {
  sha512_t s; sha512_init( &s ); sha512_append( &s, in, sz ); sha512_fini( &s, out );
}

/* ===================================================================
   GF(2^255-19), radix 2^51.  Restates the field API of
   src/ballet/ed25519/fd_f25519.h:16-25 (ref backend ref/fd_f25519.h,
   fiat-crypto 5x51): frombytes ignores bit 255 and accepts
   non-canonical y >= p (fiat-crypto/curve25519_64.c:802), tobytes is
   canonical.
   =================================================================== */

typedef struct { uint64_t v[5]; } fe;
#define M51 ((1UL<<51)-1UL)

static inline uint64_t load_le64( uint8_t const * p ) {
  uint64_t r = 0; for( int i=7; i>=0; i-- ) r = (r<<8) | p[i]; return r;
}

static void fe_frombytes( fe * h, uint8_t const s[ 32 ] ) {
  uint64_t w0 = load_le64( s ), w1 = load_le64( s+8 ), w2 = load_le64( s+16 ), w3 = load_le64( s+24 ) & 0x7fffffffffffffffUL;
  h->v[0] =  w0                  & M51;
  h->v[1] = (w0>>51 | w1<<13)    & M51;
  h->v[2] = (w1>>38 | w2<<26)    & M51;
  h->v[3] = (w2>>25 | w3<<39)    & M51;
  h->v[4] =  w3>>12;
}

static inline void fe_carry( fe * h ) {
  uint64_t c;
  c = h->v[0]>>51; h->v[0] &= M51; h->v[1] += c;
  c = h->v[1]>>51; h->v[1] &= M51; h->v[2] += c;
  c = h->v[2]>>51; h->v[2] &= M51; h->v[3] += c;
  c = h->v[3]>>51; h->v[3] &= M51; h->v[4] += c;
  c = h->v[4]>>51; h->v[4] &= M51; h->v[0] += 19*c;
  c = h->v[0]>>51; h->v[0] &= M51; h->v[1] += c;
}

static void fe_tobytes( uint8_t s[ 32 ], fe const * a ) {
  fe h = *a;
  fe_carry( &h ); fe_carry( &h );
  /* h < 2^255 + 2^13 now; subtract p if h >= p */
  uint64_t q = (h.v[0] + 19) >> 51;
  q = (h.v[1] + q) >> 51; q = (h.v[2] + q) >> 51; q = (h.v[3] + q) >> 51; q = (h.v[4] + q) >> 51;
  h.v[0] += 19*q;
  uint64_t c;
  c = h.v[0]>>51; h.v[0] &= M51; h.v[1] += c;
  c = h.v[1]>>51; h.v[1] &= M51; h.v[2] += c;
  c = h.v[2]>>51; h.v[2] &= M51; h.v[3] += c;
  c = h.v[3]>>51; h.v[3] &= M51; h.v[4] += c;
  h.v[4] &= M51;
  uint64_t w0 = h.v[0] | h.v[1]<<51, w1 = h.v[1]>>13 | h.v[2]<<38, w2 = h.v[2]>>26 | h.v[3]<<25, w3 = h.v[3]>>39 | h.v[4]<<12;
  uint64_t w[4] = { w0, w1, w2, w3 };
  for( int i=0; i<4; i++ ) for( int j=0; j<8; j++ ) s[8*i+j] = (uint8_t)(w[i] >> (8*j));
}

static inline void fe_add( fe * h, fe const * a, fe const * b ) {
  for( int i=0; i<5; i++ ) h->v[i] = a->v[i] + b->v[i];
  fe_carry( h );
}

static inline void fe_sub( fe * h, fe const * a, fe const * b ) {
  /* a + 4p - b; limbs of a,b < 2^52 after any op here */
  h->v[0] = a->v[0] + 0x1fffffffffffb4UL - b->v[0];
  for( int i=1; i<5; i++ ) h->v[i] = a->v[i] + 0x1ffffffffffffcUL - b->v[i];
  fe_carry( h );
}

static inline void fe_neg( fe * h, fe const * a ) { fe z = {{0,0,0,0,0}}; fe_sub( h, &z, a ); }

static void fe_mul( fe * h, fe const * f, fe const * g ) {
  uint64_t f0=f->v[0], f1=f->v[1], f2=f->v[2], f3=f->v[3], f4=f->v[4];
  uint64_t g0=g->v[0], g1=g->v[1], g2=g->v[2], g3=g->v[3], g4=g->v[4];
  uint64_t g1_19=19*g1, g2_19=19*g2, g3_19=19*g3, g4_19=19*g4;
  u128 r0 = (u128)f0*g0 + (u128)f1*g4_19 + (u128)f2*g3_19 + (u128)f3*g2_19 + (u128)f4*g1_19;
  u128 r1 = (u128)f0*g1 + (u128)f1*g0    + (u128)f2*g4_19 + (u128)f3*g3_19 + (u128)f4*g2_19;
  u128 r2 = (u128)f0*g2 + (u128)f1*g1    + (u128)f2*g0    + (u128)f3*g4_19 + (u128)f4*g3_19;
  u128 r3 = (u128)f0*g3 + (u128)f1*g2    + (u128)f2*g1    + (u128)f3*g0    + (u128)f4*g4_19;
  u128 r4 = (u128)f0*g4 + (u128)f1*g3    + (u128)f2*g2    + (u128)f3*g1    + (u128)f4*g0;
  uint64_t c;
  r1 += (uint64_t)(r0>>51); uint64_t h0 = (uint64_t)r0 & M51;
  r2 += (uint64_t)(r1>>51); uint64_t h1 = (uint64_t)r1 & M51;
  r3 += (uint64_t)(r2>>51); uint64_t h2 = (uint64_t)r2 & M51;
  r4 += (uint64_t)(r3>>51); uint64_t h3 = (uint64_t)r3 & M51;
  c = (uint64_t)(r4>>51);   uint64_t h4 = (uint64_t)r4 & M51;
  h0 += 19*c; c = h0>>51; h0 &= M51; h1 += c;
  h->v[0]=h0; h->v[1]=h1; h->v[2]=h2; h->v[3]=h3; h->v[4]=h4;
}

static inline void fe_sq( fe * h, fe const * f ) { fe_mul( h, f, f ); }

static inline void fe_sqn( fe * h, fe const * f, int n ) { fe_sq( h, f ); for( int i=1; i<n; i++ ) fe_sq( h, h ); }

static int fe_iszero( fe const * a ) {
  uint8_t s[32]; fe_tobytes( s, a ); uint8_t r = 0; for( int i=0; i<32; i++ ) r |= s[i]; return r==0;
}
static int fe_eq( fe const * a, fe const * b ) {
  uint8_t s[32], t[32]; fe_tobytes( s, a ); fe_tobytes( t, b ); return !memcmp( s, t, 32 );
}
static int fe_isodd( fe const * a ) { uint8_t s[32]; fe_tobytes( s, a ); return s[0]&1; }

/* a^(2^252-3); addition chain of fd_f25519.c:10-59 */
static void fe_pow22523( fe * r, fe const * a ) {
  fe t0, t1, t2;
  fe_sq( &t0, a );
  fe_sqn( &t1, &t0, 2 );
  fe_mul( &t1, a, &t1 );
  fe_mul( &t0, &t0, &t1 );
  fe_sq( &t0, &t0 );
  fe_mul( &t0, &t1, &t0 );
  fe_sqn( &t1, &t0, 5 );
  fe_mul( &t0, &t1, &t0 );
  fe_sqn( &t1, &t0, 10 );
  fe_mul( &t1, &t1, &t0 );
  fe_sqn( &t2, &t1, 20 );
  fe_mul( &t1, &t2, &t1 );
  fe_sqn( &t1, &t1, 10 );
  fe_mul( &t0, &t1, &t0 );
  fe_sqn( &t1, &t0, 50 );
  fe_mul( &t1, &t1, &t0 );
  fe_sqn( &t2, &t1, 100 );
  fe_mul( &t1, &t2, &t1 );
  fe_sqn( &t1, &t1, 50 );
  fe_mul( &t0, &t1, &t0 );
  fe_sqn( &t0, &t0, 2 );
  fe_mul( r, &t0, a );
}

/* a^(p-2) = a^(2^255-21); fd_f25519.c:62-103 */
static void fe_invert( fe * r, fe const * z ) {
  fe t0, t1, t2, t3;
  fe_sq( &t0, z );                  /* 2 */
  fe_sqn( &t1, &t0, 2 );            /* 8 */
  fe_mul( &t1, z, &t1 );            /* 9 */
  fe_mul( &t0, &t0, &t1 );          /* 11 */
  fe_sq( &t2, &t0 );                /* 22 */
  fe_mul( &t1, &t1, &t2 );          /* 2^5-1 */
  fe_sqn( &t2, &t1, 5 ); fe_mul( &t1, &t2, &t1 );    /* 2^10-1 */
  fe_sqn( &t2, &t1, 10 ); fe_mul( &t2, &t2, &t1 );   /* 2^20-1 */
  fe_sqn( &t3, &t2, 20 ); fe_mul( &t2, &t3, &t2 );   /* 2^40-1 */
  fe_sqn( &t2, &t2, 10 ); fe_mul( &t1, &t2, &t1 );   /* 2^50-1 */
  fe_sqn( &t2, &t1, 50 ); fe_mul( &t2, &t2, &t1 );   /* 2^100-1 */
  fe_sqn( &t3, &t2, 100 ); fe_mul( &t2, &t3, &t2 );  /* 2^200-1 */
  fe_sqn( &t2, &t2, 50 ); fe_mul( &t1, &t2, &t1 );   /* 2^250-1 */
  fe_sqn( &t1, &t1, 5 );                             /* 2^255-32 */
  fe_mul( r, &t1, &t0 );                             /* 2^255-21 */
}

static void fe_frombytes_hex( fe * h, char const * hex ) {
  uint8_t b[32];
  for( int i=0; i<32; i++ ) {
    int hi = hex[2*i], lo = hex[2*i+1];
    hi = hi<='9' ? hi-'0' : (hi|32)-'a'+10; lo = lo<='9' ? lo-'0' : (lo|32)-'a'+10;
    b[i] = (uint8_t)(hi<<4 | lo);
  }
  fe_frombytes( h, b );
}

/* ===================================================================
   Curve constants.  d, sqrt(-1), base point, order-8 y coordinates
   (src/ballet/ed25519/fd_curve25519.h:88-118 comment;
   table/fd_curve25519_table_*.c:17-26).  Derived at init.
   =================================================================== */

static fe fe_one, fe_d, fe_d2, fe_sqrtm1, fe_y0, fe_y1;

typedef struct { fe X, Y, Z, T; } ge_p3;      /* extended */
typedef struct { fe X, Y, Z; } ge_p2;         /* projective */
typedef struct { fe X, Y, Z, T; } ge_p1p1;    /* completed */
typedef struct { fe YpX, YmX, Z, T2d; } ge_cached;
typedef struct { fe ypx, ymx, xy2d; } ge_precomp; /* affine, Z=1 */

static ge_precomp base_odd[ 128 ]; /* [1,3,...,255] B; table/fd_curve25519_table_*.c:28-31 */
static ge_p3 base_point;
static pthread_once_t init_once = PTHREAD_ONCE_INIT;

static void ge_p3_0( ge_p3 * h ) {
  memset( h, 0, sizeof(*h) ); h->Y = fe_one; h->Z = fe_one;
}

static void p1p1_to_p2( ge_p2 * r, ge_p1p1 const * p ) {
  fe_mul( &r->X, &p->X, &p->T ); fe_mul( &r->Y, &p->Y, &p->Z ); fe_mul( &r->Z, &p->Z, &p->T );
}
static void p1p1_to_p3( ge_p3 * r, ge_p1p1 const * p ) {
  fe_mul( &r->X, &p->X, &p->T ); fe_mul( &r->Y, &p->Y, &p->Z ); fe_mul( &r->Z, &p->Z, &p->T ); fe_mul( &r->T, &p->X, &p->Y );
}

/* Doubling, a=-1 twisted Edwards (eprint 2008/522 §4.4; reference
   FD_R43X6_GE_DBL avx512/fd_r43x6_ge.h:217-236, ref/fd_curve25519.c). */
static void p2_dbl( ge_p1p1 * r, ge_p2 const * p ) {
  fe t0;
  fe_sq( &r->X, &p->X );
  fe_sq( &r->Z, &p->Y );
  fe_sq( &r->T, &p->Z ); fe_add( &r->T, &r->T, &r->T );
  fe_add( &r->Y, &p->X, &p->Y );
  fe_sq( &t0, &r->Y );
  fe_add( &r->Y, &r->Z, &r->X );
  fe_sub( &r->Z, &r->Z, &r->X );
  fe_sub( &r->X, &t0, &r->Y );
  fe_sub( &r->T, &r->T, &r->Z );
}

/* Addition with a cached point (eprint 2008/522 §4.2). */
static void p3_add_cached( ge_p1p1 * r, ge_p3 const * p, ge_cached const * q, int neg ) {
  fe a, b, c, dd, t;
  fe_add( &a, &p->Y, &p->X ); fe_sub( &b, &p->Y, &p->X );
  fe_mul( &a, &a, neg ? &q->YmX : &q->YpX );
  fe_mul( &b, &b, neg ? &q->YpX : &q->YmX );
  fe_mul( &c, &q->T2d, &p->T );
  fe_mul( &dd, &p->Z, &q->Z ); fe_add( &t, &dd, &dd );
  fe_sub( &r->X, &a, &b );
  fe_add( &r->Y, &a, &b );
  if( !neg ) { fe_add( &r->Z, &t, &c ); fe_sub( &r->T, &t, &c ); }
  else       { fe_sub( &r->Z, &t, &c ); fe_add( &r->T, &t, &c ); }
}

static void p3_add_precomp( ge_p1p1 * r, ge_p3 const * p, ge_precomp const * q, int neg ) {
  fe a, b, c, t;
  fe_add( &a, &p->Y, &p->X ); fe_sub( &b, &p->Y, &p->X );
  fe_mul( &a, &a, neg ? &q->ymx : &q->ypx );
  fe_mul( &b, &b, neg ? &q->ypx : &q->ymx );
  fe_mul( &c, &q->xy2d, &p->T );
  fe_add( &t, &p->Z, &p->Z );
  fe_sub( &r->X, &a, &b );
  fe_add( &r->Y, &a, &b );
  if( !neg ) { fe_add( &r->Z, &t, &c ); fe_sub( &r->T, &t, &c ); }
  else       { fe_sub( &r->Z, &t, &c ); fe_add( &r->T, &t, &c ); }
}

static void p3_to_cached( ge_cached * r, ge_p3 const * p ) {
  fe_add( &r->YpX, &p->Y, &p->X ); fe_sub( &r->YmX, &p->Y, &p->X ); r->Z = p->Z; fe_mul( &r->T2d, &p->T, &fe_d2 );
}

static void p3_add( ge_p3 * r, ge_p3 const * p, ge_p3 const * q ) {
  ge_cached c; ge_p1p1 t; p3_to_cached( &c, q ); p3_add_cached( &t, p, &c, 0 ); p1p1_to_p3( r, &t );
}

static void p3_dbl( ge_p3 * r, ge_p3 const * p ) {
  ge_p2 q = { p->X, p->Y, p->Z }; ge_p1p1 t; p2_dbl( &t, &q ); p1p1_to_p3( r, &t );
}

/* ===================================================================
   Point decoding.  Restates fd_ed25519_point_frombytes
   (fd_curve25519.c:22-49, fd_f25519_sqrt_ratio fd_f25519.c:105-143)
   with the AVX-512 decode rule of FD_R43X6_GE_DECODE2
   (avx512/fd_r43x6_ge.c:163-254): x==0 with sign bit set is rejected.
   =================================================================== */

static int ge_decode( ge_p3 * P, uint8_t const enc[ 32 ], int semantics ) {
  fe y, u, v, v3, uv3, v7, uv7, x, vx2, t, nu;
  fe_frombytes( &y, enc );
  int sign = enc[31] >> 7;
  fe_sq( &u, &y );
  fe_mul( &v, &u, &fe_d );
  fe_sub( &u, &u, &fe_one );   /* u = y^2-1 */
  fe_add( &v, &v, &fe_one );   /* v = dy^2+1 */
  fe_sq( &v3, &v ); fe_mul( &v3, &v3, &v );
  fe_mul( &uv3, &u, &v3 );
  fe_sq( &v7, &v3 ); fe_mul( &v7, &v7, &v );
  fe_mul( &uv7, &u, &v7 );
  fe_pow22523( &t, &uv7 );
  fe_mul( &x, &uv3, &t );
  fe_sq( &vx2, &x ); fe_mul( &vx2, &vx2, &v );
  fe_neg( &nu, &u );
  if( fe_eq( &vx2, &u ) ) { /* correct sign sqrt */ }
  else if( fe_eq( &vx2, &nu ) ) { fe_mul( &x, &x, &fe_sqrtm1 ); }
  else return 1; /* not a square */
  int x_is_zero = fe_iszero( &x );
  if( x_is_zero && sign && semantics==FDGPU_SEMANTICS_AVX512 ) return 2;
  if( fe_isodd( &x ) != sign ) fe_neg( &x, &x );
  P->X = x; P->Y = y; P->Z = fe_one; fe_mul( &P->T, &x, &y );
  return 0;
}

/* fd_ed25519_affine_is_small_order, fd_curve25519.h:88-118 */
static int ge_affine_is_small_order( ge_p3 const * P ) {
  return fe_iszero( &P->X ) | fe_iszero( &P->Y ) | fe_eq( &P->Y, &fe_y0 ) | fe_eq( &P->Y, &fe_y1 );
}

static void ge_encode( uint8_t out[ 32 ], ge_p3 const * P ) {
  fe zi, x, y; fe_invert( &zi, &P->Z ); fe_mul( &x, &P->X, &zi ); fe_mul( &y, &P->Y, &zi );
  fe_tobytes( out, &y ); out[31] ^= (uint8_t)(fe_isodd( &x ) << 7);
}

static void oracle_init( void ) {
  memset( &fe_one, 0, sizeof(fe) ); fe_one.v[0] = 1;
  fe n, dd; memset( &n, 0, sizeof(fe) ); n.v[0] = 121666; fe_invert( &dd, &n );
  memset( &n, 0, sizeof(fe) ); n.v[0] = 121665; fe_mul( &dd, &dd, &n ); fe_neg( &fe_d, &dd );
  fe_add( &fe_d2, &fe_d, &fe_d );
  fe_frombytes_hex( &fe_sqrtm1, "b0a00e4a271beec478e42fad0618432fa7d7fb3d99004d2b0bdfc14f8024832b" );
  fe_frombytes_hex( &fe_y0, "26e8958fc2b227b045c3f489f2ef98f0d5dfac05d3c63339b13802886d53fc05" );
  fe_frombytes_hex( &fe_y1, "c7176a703d4dd84fba3c0b760d10670f2a2053fa2c39ccc64ec7fd7792ac037a" );
  uint8_t benc[32]; memset( benc, 0x66, 32 ); benc[0] = 0x58;
  if( ge_decode( &base_point, benc, FDGPU_SEMANTICS_AVX512 ) ) __builtin_trap();
  ge_p3 b2, cur; p3_dbl( &b2, &base_point ); cur = base_point;
  for( int i=0; i<128; i++ ) {
    fe zi, x, y; fe_invert( &zi, &cur.Z ); fe_mul( &x, &cur.X, &zi ); fe_mul( &y, &cur.Y, &zi );
    fe_add( &base_odd[i].ypx, &y, &x ); fe_sub( &base_odd[i].ymx, &y, &x );
    fe_mul( &base_odd[i].xy2d, &x, &y ); fe_mul( &base_odd[i].xy2d, &base_odd[i].xy2d, &fe_d2 );
    p3_add( &cur, &cur, &b2 );
  }
}

/* ===================================================================
   Scalars mod l = 2^252 + 27742317777372353535851937790883648493.
   =================================================================== */

/* fd_curve25519_scalar_validate, fd_curve25519_scalar.h:57-73: S <= l-1 */
int oracle_scalar_validate( uint8_t const s[ 32 ] ) {
  static uint8_t const lm1[32] = {
    0xec,0xd3,0xf5,0x5c,0x1a,0x63,0x12,0x58,0xd6,0x9c,0xf7,0xa2,0xde,0xf9,0xde,0x14,
    0,0,0,0,0,0,0,0,0,0,0,0,0,0,0,0x10 };
  for( int i=31; i>=0; i-- ) { if( s[i] < lm1[i] ) return 1; if( s[i] > lm1[i] ) return 0; }
  return 1;
}

static int64_t get21( uint8_t const * s, int bit, int nbits ) {
  uint64_t w = 0; int byte = bit>>3;
  for( int i=0; i<5 && byte+i<64; i++ ) w |= (uint64_t)s[byte+i] << (8*i);
  return (int64_t)((w >> (bit&7)) & ((1UL<<nbits)-1UL));
}

/* 512-bit -> mod l in 21-bit signed limbs; the folding schedule of
   fd_curve25519_scalar_reduce (fd_curve25519_scalar.c:3-110), with
   2^252 == -c and -c in 21-bit signed digits. */
static void fold( int64_t * t, int j ) {
  int64_t v = t[j];
  t[j-12] += v * 666643; t[j-11] += v * 470296; t[j-10] += v * 654183;
  t[j- 9] -= v * 997805; t[j- 8] += v * 136657; t[j- 7] -= v * 683901;
  t[j] = 0;
}
static void carry_round( int64_t * t, int i ) { int64_t c = (t[i] + (1L<<20)) >> 21; t[i+1] += c; t[i] -= c * (1L<<21); }
static void carry_floor( int64_t * t, int i ) { int64_t c = t[i] >> 21; t[i+1] += c; t[i] -= c * (1L<<21); }

void oracle_scalar_reduce( uint8_t out[ 32 ], uint8_t const in[ 64 ] ) {
  int64_t t[25];
  for( int i=0; i<23; i++ ) t[i] = get21( in, 21*i, 21 );
  t[23] = get21( in, 483, 29 ); t[24] = 0;
  for( int j=23; j>=18; j-- ) fold( t, j );
  for( int i=6; i<=16; i+=2 ) carry_round( t, i );
  for( int i=7; i<=15; i+=2 ) carry_round( t, i );
  for( int j=17; j>=12; j-- ) fold( t, j );
  for( int i=0; i<=10; i+=2 ) carry_round( t, i );
  for( int i=1; i<=11; i+=2 ) carry_round( t, i );
  fold( t, 12 );
  for( int i=0; i<=11; i++ ) carry_floor( t, i );
  fold( t, 12 );
  for( int i=0; i<=10; i++ ) carry_floor( t, i );
  /* pack 12 limbs (t[11] may carry bit 252) */
  u128 acc = 0; int accb = 0, o = 0;
  for( int i=0; i<12; i++ ) {
    acc |= (u128)(uint64_t)t[i] << accb; accb += 21;
    while( accb >= 8 && o < 32 ) { out[o++] = (uint8_t)acc; acc >>= 8; accb -= 8; }
  }
  while( o < 32 ) { out[o++] = (uint8_t)acc; acc >>= 8; }
}

/* Sliding-window NAF, fd_curve25519_scalar_wnaf
   (fd_curve25519_scalar.c:277-360): odd digits in [-(2^bits-1), 2^bits-1]. */
static void scalar_wnaf( int16_t r[ 256 ], uint8_t const s[ 32 ], int bits ) {
  int max = (1<<bits) - 1;
  for( int i=0; i<255; i++ ) r[i] = (int16_t)((s[i>>3] >> (i&7)) & 1);
  r[255] = 0;
  for( int i=0; i<256; i++ ) {
    if( !r[i] ) continue;
    for( int b=1; b<=bits+1 && i+b<256; b++ ) {
      if( !r[i+b] ) continue;
      int v = r[i+b] << b;
      if( r[i] + v <= max ) { r[i] = (int16_t)(r[i] + v); r[i+b] = 0; }
      else if( r[i] - v >= -max ) {
        r[i] = (int16_t)(r[i] - v);
        for( int k=i+b; k<256; k++ ) { if( !r[k] ) { r[k] = 1; break; } r[k] = 0; }
      } else break;
    }
  }
}

/* fd_ed25519_double_scalar_mul_base (fd_curve25519.c:109-153):
   R = [n1]a + [n2]B, wNAF w=4 for n1 over an 8-entry odd-multiple
   table of a, w=8 for n2 over the 128-entry base table. */
static void ge_double_scalar_mul_base( ge_p2 * r, uint8_t const n1[ 32 ], ge_p3 const * a, uint8_t const n2[ 32 ] ) {
  int16_t s1[256], s2[256];
  scalar_wnaf( s1, n1, 4 ); scalar_wnaf( s2, n2, 8 );
  ge_cached ai[8]; ge_p3 a2, cur = *a;
  p3_dbl( &a2, a );
  for( int i=0; i<8; i++ ) { p3_to_cached( &ai[i], &cur ); p3_add( &cur, &cur, &a2 ); }
  memset( r, 0, sizeof(*r) ); r->Y = fe_one; r->Z = fe_one;
  int i; for( i=255; i>=0; i-- ) if( s1[i] || s2[i] ) break;
  for( ; i>=0; i-- ) {
    ge_p1p1 t; ge_p3 u;
    p2_dbl( &t, r );
    if( s1[i] ) { p1p1_to_p3( &u, &t ); p3_add_cached( &t, &u, &ai[ (s1[i]>0 ? s1[i] : -s1[i])/2 ], s1[i]<0 ); }
    if( s2[i] ) { p1p1_to_p3( &u, &t ); p3_add_precomp( &t, &u, &base_odd[ (s2[i]>0 ? s2[i] : -s2[i])/2 ], s2[i]<0 ); }
    p1p1_to_p2( r, &t );
  }
}

/* fd_ed25519_point_eq_z1 (fd_ed25519_user.c:219-229; ref/fd_curve25519.h:133-139):
   projective compare against an affine (Z=1) point. */
static int ge_eq_z1( ge_p2 const * a, ge_p3 const * b ) {
  fe t;
  fe_mul( &t, &b->X, &a->Z ); if( !fe_eq( &t, &a->X ) ) return 0;
  fe_mul( &t, &b->Y, &a->Z ); if( !fe_eq( &t, &a->Y ) ) return 0;
  return 1;
}

/* ===================================================================
   Verify.  fd_ed25519_verify (fd_ed25519_user.c:135-230) and
   fd_ed25519_verify_batch_single_msg (fd_ed25519_user.c:232-310).
   =================================================================== */

typedef struct { ge_p3 A, R; uint8_t k[32]; } pass1_t;

/* pass 1 for one signature; returns 0 or a FD_ED25519_ERR_* code */
static int verify_pass1( pass1_t * st, uint8_t const * msg, size_t msg_sz,
                         uint8_t const sig[ 64 ], uint8_t const pub[ 32 ], int semantics ) {
  uint8_t const * r = sig; uint8_t const * S = sig + 32;
  if( !oracle_scalar_validate( S ) ) return FD_ED25519_ERR_SIG;
  /* fd_ed25519_point_frombytes_2x( A, pub, R, r ); AVX-512: any failure
     -> res<0 -> ERR_SIG (fd_r43x6_ge.c:241-251 + fd_ed25519_user.c:191-193);
     ref: A failure -> 1 -> ERR_PUBKEY, R failure -> 2 -> ERR_SIG
     (ref/fd_curve25519.c:209-224). */
  int ra = ge_decode( &st->A, pub, semantics );
  if( semantics==FDGPU_SEMANTICS_AVX512 ) {
    int rr = ge_decode( &st->R, r, semantics );
    if( ra || rr ) return FD_ED25519_ERR_SIG;
  } else {
    if( ra ) return FD_ED25519_ERR_PUBKEY;
    if( ge_decode( &st->R, r, semantics ) ) return FD_ED25519_ERR_SIG;
  }
  if( ge_affine_is_small_order( &st->A ) ) return FD_ED25519_ERR_PUBKEY;
  if( ge_affine_is_small_order( &st->R ) ) return FD_ED25519_ERR_SIG;
  sha512_t sh; uint8_t h[64];
  sha512_init( &sh ); sha512_append( &sh, r, 32 ); sha512_append( &sh, pub, 32 ); sha512_append( &sh, msg, msg_sz );
  sha512_fini( &sh, h );
  oracle_scalar_reduce( st->k, h );
  return 0;
}

static int verify_pass2( pass1_t * st, uint8_t const S[ 32 ] ) {
  ge_p3 negA = st->A;
  fe_neg( &negA.X, &negA.X ); fe_neg( &negA.T, &negA.T );   /* fd_ed25519_point_neg */
  ge_p2 Rc;
  ge_double_scalar_mul_base( &Rc, st->k, &negA, S );
  return ge_eq_z1( &Rc, &st->R ) ? FD_ED25519_SUCCESS : FD_ED25519_ERR_MSG;
}

int oracle_ed25519_verify( uint8_t const * msg, size_t msg_sz,
                           uint8_t const sig[ 64 ], uint8_t const pub[ 32 ], int semantics ) {
  pthread_once( &init_once, oracle_init );
  pass1_t st;
  int rc = verify_pass1( &st, msg, msg_sz, sig, pub, semantics );
  if( rc ) return rc;
  return verify_pass2( &st, sig+32 );
}

int oracle_ed25519_verify_batch_single_msg( uint8_t const * msg, size_t msg_sz,
                                            uint8_t const * sigs, uint8_t const * pubs,
                                            uint8_t batch_sz, int semantics ) {
  pthread_once( &init_once, oracle_init );
  if( batch_sz==0 || batch_sz>16 ) return FD_ED25519_ERR_SIG;
  pass1_t st[16];
  for( int j=0; j<batch_sz; j++ ) {
    int rc = verify_pass1( &st[j], msg, msg_sz, sigs + 64*j, pubs + 32*j, semantics );
    if( rc ) return rc;
  }
  for( int j=0; j<batch_sz; j++ ) {
    if( verify_pass2( &st[j], sigs + 64*j + 32 ) ) return FD_ED25519_ERR_MSG;
  }
  return FD_ED25519_SUCCESS;
}

int oracle_point_decode( uint8_t x[ 32 ], uint8_t y[ 32 ], uint8_t const enc[ 32 ], int semantics ) {
  pthread_once( &init_once, oracle_init );
  ge_p3 P; int rc = ge_decode( &P, enc, semantics );
  if( rc ) return rc;
  fe_tobytes( x, &P.X ); fe_tobytes( y, &P.Y );
  return 0;
}

int oracle_dsm_encode( uint8_t out[ 32 ], uint8_t const k[ 32 ], uint8_t const A[ 32 ], uint8_t const S[ 32 ] ) {
  pthread_once( &init_once, oracle_init );
  ge_p3 a; if( ge_decode( &a, A, FDGPU_SEMANTICS_REF ) ) return -1;
  fe_neg( &a.X, &a.X ); fe_neg( &a.T, &a.T );
  ge_p2 r; ge_double_scalar_mul_base( &r, k, &a, S );
  ge_p3 r3 = { r.X, r.Y, r.Z, r.Z };
  ge_encode( out, &r3 );
  return 0;
}

/* ===================================================================
   Batch layout (include/fd_ed25519_gpu.h fdgpu_txn_desc_t), per
   fd_txn_verify (src/disco/verify/fd_verify_tile.h:59-108).
   =================================================================== */

static int txn_bounds_ok( fdgpu_txn_desc_t const * d ) {
  unsigned n = d->sig_cnt;
  if( n==0 || n>16 ) return 0;
  if( (unsigned)d->signature_off + 64u*n > d->payload_sz ) return 0;
  if( (unsigned)d->acct_addr_off + 32u*n > d->payload_sz ) return 0;
  if( d->message_off > d->payload_sz ) return 0;
  return 1;
}

static void verify_txn( uint8_t const * payload, fdgpu_txn_desc_t const * d, int8_t * txn_out, int8_t * sig_out, int semantics ) {
  uint8_t const * base = payload + d->payload_off;
  if( !txn_bounds_ok( d ) ) {
    *txn_out = FD_ED25519_ERR_SIG;
    if( sig_out ) for( unsigned j=0; j<d->sig_cnt; j++ ) sig_out[ d->sig_base + j ] = FD_ED25519_ERR_SIG;
    return;
  }
  uint8_t const * msg = base + d->message_off; size_t msg_sz = (size_t)d->payload_sz - d->message_off;
  int first = 0, any_msg = 0;
  for( unsigned j=0; j<d->sig_cnt; j++ ) {
    int rc = oracle_ed25519_verify( msg, msg_sz, base + d->signature_off + 64*j, base + d->acct_addr_off + 32*j, semantics );
    if( sig_out ) sig_out[ d->sig_base + j ] = (int8_t)rc;
    if( rc==FD_ED25519_ERR_MSG ) any_msg = 1;
    else if( rc && !first ) first = rc;
  }
  *txn_out = (int8_t)( first ? first : ( any_msg ? FD_ED25519_ERR_MSG : FD_ED25519_SUCCESS ) );
}

typedef struct {
  uint8_t const * payload; fdgpu_txn_desc_t const * desc; size_t lo, hi;
  int8_t * txn_out; int8_t * sig_out; int semantics;
} job_t;

static void * job_run( void * _j ) {
  job_t * j = (job_t *)_j;
  for( size_t i=j->lo; i<j->hi; i++ ) verify_txn( j->payload, j->desc + i, j->txn_out + i, j->sig_out, j->semantics );
  return NULL;
}

void oracle_verify_txns( uint8_t const * payload, fdgpu_txn_desc_t const * desc, size_t txn_cnt,
                         int8_t * txn_out, int8_t * sig_out, int semantics, int threads ) {
  pthread_once( &init_once, oracle_init );
  if( threads < 1 ) threads = 1;
  if( threads > 256 ) threads = 256;
  pthread_t th[256]; job_t jobs[256];
  for( int t=0; t<threads; t++ ) {
    jobs[t] = (job_t){ payload, desc, txn_cnt*(size_t)t/(size_t)threads, txn_cnt*(size_t)(t+1)/(size_t)threads, txn_out, sig_out, semantics };
    if( t ) pthread_create( &th[t], NULL, job_run, &jobs[t] );
  }
  job_run( &jobs[0] );
  for( int t=1; t<threads; t++ ) pthread_join( th[t], NULL );
}

/* ===================================================================
   Test-data helpers: RFC 8032 key generation and signing
   (fd_ed25519_user.c:4-133 restated; not constant time).
   =================================================================== */

static void ge_scalarmult_base( ge_p3 * r, uint8_t const s[ 32 ] ) {
  ge_p3_0( r );
  for( int i=255; i>=0; i-- ) {
    p3_dbl( r, r );
    if( (s[i>>3] >> (i&7)) & 1 ) p3_add( r, r, &base_point );
  }
}

void oracle_ed25519_public_from_private( uint8_t pub[ 32 ], uint8_t const prv[ 32 ] ) {
  pthread_once( &init_once, oracle_init );
  uint8_t h[64]; oracle_sha512( prv, 32, h );
  h[0] &= 0xf8; h[31] &= 0x7f; h[31] |= 0x40;
  ge_p3 A; ge_scalarmult_base( &A, h ); ge_encode( pub, &A );
}

static void sc_muladd( uint8_t s[ 32 ], uint8_t const a[ 32 ], uint8_t const b[ 32 ], uint8_t const c[ 32 ] ) {
  /* (a*b + c) mod l via schoolbook into 512 bits then reduce */
  uint32_t prod[17] = {0}; uint8_t wide[64];
  uint64_t aw[8], bw[8];
  for( int i=0; i<8; i++ ) { aw[i] = (uint64_t)a[4*i] | (uint64_t)a[4*i+1]<<8 | (uint64_t)a[4*i+2]<<16 | (uint64_t)a[4*i+3]<<24;
                             bw[i] = (uint64_t)b[4*i] | (uint64_t)b[4*i+1]<<8 | (uint64_t)b[4*i+2]<<16 | (uint64_t)b[4*i+3]<<24; }
  uint64_t cw[16] = {0};
  for( int i=0; i<8; i++ ) cw[i] = (uint64_t)c[4*i] | (uint64_t)c[4*i+1]<<8 | (uint64_t)c[4*i+2]<<16 | (uint64_t)c[4*i+3]<<24;
  u128 acc = 0;
  for( int k=0; k<16; k++ ) {
    u128 col = acc;
    for( int i=0; i<8; i++ ) { int j = k-i; if( j<0 || j>7 ) continue; col += (u128)aw[i]*bw[j]; }
    col += cw[k];
    prod[k] = (uint32_t)col; acc = col >> 32;
  }
  for( int k=0; k<16; k++ ) for( int j=0; j<4; j++ ) wide[4*k+j] = (uint8_t)(prod[k] >> (8*j));
  oracle_scalar_reduce( s, wide );
}

void oracle_ed25519_sign( uint8_t sig[ 64 ], uint8_t const * msg, size_t msg_sz,
                          uint8_t const pub[ 32 ], uint8_t const prv[ 32 ] ) {
  pthread_once( &init_once, oracle_init );
  uint8_t h[64]; oracle_sha512( prv, 32, h );
  h[0] &= 0xf8; h[31] &= 0x7f; h[31] |= 0x40;
  sha512_t sh; uint8_t r[64], rr[32], k[64], kk[32];
  sha512_init( &sh ); sha512_append( &sh, h+32, 32 ); sha512_append( &sh, msg, msg_sz ); sha512_fini( &sh, r );
  oracle_scalar_reduce( rr, r );
  ge_p3 R; ge_scalarmult_base( &R, rr ); ge_encode( sig, &R );
  sha512_init( &sh ); sha512_append( &sh, sig, 32 ); sha512_append( &sh, pub, 32 ); sha512_append( &sh, msg, msg_sz ); sha512_fini( &sh, k );
  oracle_scalar_reduce( kk, k );
  sc_muladd( sig+32, kk, h, rr );
}
