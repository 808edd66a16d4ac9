/* fd_synth.c -- synthetic signed Solana transactions for benches/tests.

   Host C, independent of the verify engine and of oracle/.  The
   transaction layout follows the reference's synthetic load generator
   (src/app/shared_dev/commands/bench/fd_benchg.c:102-171,309-314):
   a 1232-byte "large_noop" txn has sig_cnt=1 at byte 0, the signature at
   bytes 1..64 and signs bytes 65..1231 (1167 bytes); the fee payer
   pubkey (account 0) is at byte 69.  Multi-signer transactions use the
   same wire format with n signatures and n signer accounts first.

   Signing: RFC 8032 (5.1.6) with a radix-16 fixed-base comb for [r]B
   (64 affine table adds); GF(2^255-19) in radix 2^51.  Not constant time
   -- test data only. */

#include "../../include/fd_ed25519_gpu.h"
#include <stdint.h>
#include <string.h>
#include <pthread.h>

typedef unsigned __int128 u128;

/* ---- SHA-512 ---------------------------------------------------------- */

static const uint64_t K[80] = {
  0x428a2f98d728ae22UL,0x7137449123ef65cdUL,0xb5c0fbcfec4d3b2fUL,0xe9b5dba58189dbbcUL,0x3956c25bf348b538UL,
  0x59f111f1b605d019UL,0x923f82a4af194f9bUL,0xab1c5ed5da6d8118UL,0xd807aa98a3030242UL,0x12835b0145706fbeUL,
  0x243185be4ee4b28cUL,0x550c7dc3d5ffb4e2UL,0x72be5d74f27b896fUL,0x80deb1fe3b1696b1UL,0x9bdc06a725c71235UL,
  0xc19bf174cf692694UL,0xe49b69c19ef14ad2UL,0xefbe4786384f25e3UL,0x0fc19dc68b8cd5b5UL,0x240ca1cc77ac9c65UL,
  0x2de92c6f592b0275UL,0x4a7484aa6ea6e483UL,0x5cb0a9dcbd41fbd4UL,0x76f988da831153b5UL,0x983e5152ee66dfabUL,
  0xa831c66d2db43210UL,0xb00327c898fb213fUL,0xbf597fc7beef0ee4UL,0xc6e00bf33da88fc2UL,0xd5a79147930aa725UL,
  0x06ca6351e003826fUL,0x142929670a0e6e70UL,0x27b70a8546d22ffcUL,0x2e1b21385c26c926UL,0x4d2c6dfc5ac42aedUL,
  0x53380d139d95b3dfUL,0x650a73548baf63deUL,0x766a0abb3c77b2a8UL,0x81c2c92e47edaee6UL,0x92722c851482353bUL,
  0xa2bfe8a14cf10364UL,0xa81a664bbc423001UL,0xc24b8b70d0f89791UL,0xc76c51a30654be30UL,0xd192e819d6ef5218UL,
  0xd69906245565a910UL,0xf40e35855771202aUL,0x106aa07032bbd1b8UL,0x19a4c116b8d2d0c8UL,0x1e376c085141ab53UL,
  0x2748774cdf8eeb99UL,0x34b0bcb5e19b48a8UL,0x391c0cb3c5c95a63UL,0x4ed8aa4ae3418acbUL,0x5b9cca4f7763e373UL,
  0x682e6ff3d6b2b8a3UL,0x748f82ee5defb2fcUL,0x78a5636f43172f60UL,0x84c87814a1f0ab72UL,0x8cc702081a6439ecUL,
  0x90befffa23631e28UL,0xa4506cebde82bde9UL,0xbef9a3f7b2c67915UL,0xc67178f2e372532bUL,0xca273eceea26619cUL,
  0xd186b8c721c0c207UL,0xeada7dd6cde0eb1eUL,0xf57d4f7fee6ed178UL,0x06f067aa72176fbaUL,0x0a637dc5a2c898a6UL,
  0x113f9804bef90daeUL,0x1b710b35131c471bUL,0x28db77f523047d84UL,0x32caab7b40c72493UL,0x3c9ebe0a15c9bebcUL,
  0x431d67c49c100d4cUL,0x4cc5d4becb3e42b6UL,0x597f299cfc657e2aUL,0x5fcb6fab3ad6faecUL,0x6c44198c4a475817UL };

#define ROR(x,n) (((x)>>(n))|((x)<<(64-(n))))

typedef struct { uint64_t h[8]; uint8_t b[128]; size_t n; uint64_t len; } sha_t;

static void sha_blk( uint64_t * h, uint8_t const * p ) {
  uint64_t w[80];
  for( int i=0; i<16; i++ ) { uint64_t x = 0; for( int j=0; j<8; j++ ) x = x<<8 | p[8*i+j]; w[i] = x; }
  for( int i=16; i<80; i++ ) w[i] = w[i-16] + (ROR(w[i-15],1)^ROR(w[i-15],8)^(w[i-15]>>7)) + w[i-7] + (ROR(w[i-2],19)^ROR(w[i-2],61)^(w[i-2]>>6));
  uint64_t a=h[0],b=h[1],c=h[2],d=h[3],e=h[4],f=h[5],g=h[6],k=h[7];
  for( int i=0; i<80; i++ ) {
    uint64_t t1 = k + (ROR(e,14)^ROR(e,18)^ROR(e,41)) + ((e&f)^(~e&g)) + K[i] + w[i];
    uint64_t t2 = (ROR(a,28)^ROR(a,34)^ROR(a,39)) + ((a&b)^(a&c)^(b&c));
    k=g; g=f; f=e; e=d+t1; d=c; c=b; b=a; a=t1+t2;
  }
  h[0]+=a; h[1]+=b; h[2]+=c; h[3]+=d; h[4]+=e; h[5]+=f; h[6]+=g; h[7]+=k;
}
static void sha_init( sha_t * s ) {
  static const uint64_t iv[8] = { 0x6a09e667f3bcc908UL,0xbb67ae8584caa73bUL,0x3c6ef372fe94f82bUL,0xa54ff53a5f1d36f1UL,
                                  0x510e527fade682d1UL,0x9b05688c2b3e6c1fUL,0x1f83d9abfb41bd6bUL,0x5be0cd19137e2179UL };
  memcpy( s->h, iv, 64 ); s->n = 0; s->len = 0;
}
static void sha_add( sha_t * s, uint8_t const * p, size_t n ) {
  s->len += n;
  if( s->n ) { size_t k = 128 - s->n; if( k > n ) k = n; memcpy( s->b + s->n, p, k ); s->n += k; p += k; n -= k;
               if( s->n==128 ) { sha_blk( s->h, s->b ); s->n = 0; } }
  while( n >= 128 ) { sha_blk( s->h, p ); p += 128; n -= 128; }
  if( n ) { memcpy( s->b, p, n ); s->n = n; }
}
static void sha_fin( sha_t * s, uint8_t out[64] ) {
  uint64_t bits = s->len << 3;
  uint8_t pad[144] = { 0x80 };
  size_t k = (s->n < 112) ? 112 - s->n : 240 - s->n;
  for( int i=0; i<8; i++ ) pad[k+8+i] = (uint8_t)(bits >> (56-8*i));
  sha_add( s, pad, k+16 );
  for( int i=0; i<8; i++ ) for( int j=0; j<8; j++ ) out[8*i+j] = (uint8_t)(s->h[i] >> (56-8*j));
}

/* ---- field 2^255-19, radix 2^51 ----------------------------------------- */

typedef struct { uint64_t v[5]; } f;
#define M51 ((1UL<<51)-1)

static void f_carry( f * h ) {
  uint64_t c;
  for( int i=0; i<4; i++ ) { c = h->v[i]>>51; h->v[i] &= M51; h->v[i+1] += c; }
  c = h->v[4]>>51; h->v[4] &= M51; h->v[0] += 19*c;
  c = h->v[0]>>51; h->v[0] &= M51; h->v[1] += c;
}
static void f_add( f * r, f const * a, f const * b ) { for( int i=0; i<5; i++ ) r->v[i] = a->v[i] + b->v[i]; f_carry( r ); }
static void f_sub( f * r, f const * a, f const * b ) {
  r->v[0] = a->v[0] + 0x1fffffffffffb4UL - b->v[0];
  for( int i=1; i<5; i++ ) r->v[i] = a->v[i] + 0x1ffffffffffffcUL - b->v[i];
  f_carry( r );
}
static void f_mul( f * r, f const * a, f const * b ) {
  u128 t[5] = {0};
  for( int i=0; i<5; i++ ) for( int j=0; j<5; j++ ) {
    u128 p = (u128)a->v[i] * b->v[j];
    if( i+j < 5 ) t[i+j] += p; else t[i+j-5] += p * 19;
  }
  uint64_t c = 0;
  for( int i=0; i<5; i++ ) { t[i] += c; r->v[i] = (uint64_t)t[i] & M51; c = (uint64_t)(t[i] >> 51); }
  r->v[0] += 19*c; f_carry( r );
}
static void f_sqn( f * r, f const * a, int n ) { f_mul( r, a, a ); for( int i=1; i<n; i++ ) f_mul( r, r, r ); }
static void f_inv( f * r, f const * z ) {
  f t0, t1, t2, t3;
  f_mul( &t0, z, z ); f_sqn( &t1, &t0, 2 ); f_mul( &t1, z, &t1 ); f_mul( &t0, &t0, &t1 );
  f_mul( &t2, &t0, &t0 ); f_mul( &t1, &t1, &t2 );
  f_sqn( &t2, &t1, 5 ); f_mul( &t1, &t2, &t1 ); f_sqn( &t2, &t1, 10 ); f_mul( &t2, &t2, &t1 );
  f_sqn( &t3, &t2, 20 ); f_mul( &t2, &t3, &t2 ); f_sqn( &t2, &t2, 10 ); f_mul( &t1, &t2, &t1 );
  f_sqn( &t2, &t1, 50 ); f_mul( &t2, &t2, &t1 ); f_sqn( &t3, &t2, 100 ); f_mul( &t2, &t3, &t2 );
  f_sqn( &t2, &t2, 50 ); f_mul( &t1, &t2, &t1 ); f_sqn( &t1, &t1, 5 ); f_mul( r, &t1, &t0 );
}
static void f_from( f * h, uint8_t const s[32] ) {
  uint64_t w[4]; for( int i=0; i<4; i++ ) { w[i] = 0; for( int j=7; j>=0; j-- ) w[i] = w[i]<<8 | s[8*i+j]; }
  w[3] &= 0x7fffffffffffffffUL;
  h->v[0] = w[0] & M51; h->v[1] = (w[0]>>51 | w[1]<<13) & M51; h->v[2] = (w[1]>>38 | w[2]<<26) & M51;
  h->v[3] = (w[2]>>25 | w[3]<<39) & M51; h->v[4] = w[3]>>12;
}
static void f_to( uint8_t s[32], f const * a ) {
  f h = *a; f_carry( &h ); f_carry( &h );
  uint64_t q = (h.v[0]+19)>>51; for( int i=1; i<5; i++ ) q = (h.v[i]+q)>>51;
  h.v[0] += 19*q;
  for( int i=0; i<4; i++ ) { h.v[i+1] += h.v[i]>>51; h.v[i] &= M51; }
  h.v[4] &= M51;
  uint64_t w[4] = { h.v[0] | h.v[1]<<51, h.v[1]>>13 | h.v[2]<<38, h.v[2]>>26 | h.v[3]<<25, h.v[3]>>39 | h.v[4]<<12 };
  for( int i=0; i<4; i++ ) for( int j=0; j<8; j++ ) s[8*i+j] = (uint8_t)(w[i]>>(8*j));
}

/* ---- points --------------------------------------------------------------- */

typedef struct { f X, Y, Z, T; } pt;
typedef struct { f ypx, ymx, xy2d; } aff;

static f F_D2;       /* 2d */
static aff comb[64][9]; /* comb[i][j] = j*16^i*B, j=0..8 */
static pthread_once_t once = PTHREAD_ONCE_INIT;

static void pt_add( pt * r, pt const * p, pt const * q ) {
  f a, b, c, d, e, ff, g, h, t;
  f_sub( &a, &p->Y, &p->X ); f_sub( &t, &q->Y, &q->X ); f_mul( &a, &a, &t );
  f_add( &b, &p->Y, &p->X ); f_add( &t, &q->Y, &q->X ); f_mul( &b, &b, &t );
  f_mul( &c, &p->T, &q->T ); f_mul( &c, &c, &F_D2 );
  f_mul( &d, &p->Z, &q->Z ); f_add( &d, &d, &d );
  f_sub( &e, &b, &a ); f_sub( &ff, &d, &c ); f_add( &g, &d, &c ); f_add( &h, &b, &a );
  f_mul( &r->X, &e, &ff ); f_mul( &r->Y, &g, &h ); f_mul( &r->Z, &ff, &g ); f_mul( &r->T, &e, &h );
}
static void pt_madd( pt * r, pt const * p, aff const * q, int neg ) {
  f a, b, c, d, e, ff, g, h;
  f_sub( &a, &p->Y, &p->X ); f_mul( &a, &a, neg ? &q->ypx : &q->ymx );
  f_add( &b, &p->Y, &p->X ); f_mul( &b, &b, neg ? &q->ymx : &q->ypx );
  f_mul( &c, &p->T, &q->xy2d ); if( neg ) { f z = {{0}}; f_sub( &c, &z, &c ); }
  f_add( &d, &p->Z, &p->Z );
  f_sub( &e, &b, &a ); f_sub( &ff, &d, &c ); f_add( &g, &d, &c ); f_add( &h, &b, &a );
  f_mul( &r->X, &e, &ff ); f_mul( &r->Y, &g, &h ); f_mul( &r->Z, &ff, &g ); f_mul( &r->T, &e, &h );
}
static void pt_zero( pt * p ) { memset( p, 0, sizeof(*p) ); p->Y.v[0] = 1; p->Z.v[0] = 1; }
static void pt_enc( uint8_t out[32], pt const * p ) {
  f zi, x, y; f_inv( &zi, &p->Z ); f_mul( &x, &p->X, &zi ); f_mul( &y, &p->Y, &zi );
  uint8_t xs[32]; f_to( xs, &x ); f_to( out, &y ); out[31] ^= (uint8_t)((xs[0]&1) << 7);
}
static void to_aff( aff * a, pt const * p ) {
  f zi, x, y; f_inv( &zi, &p->Z ); f_mul( &x, &p->X, &zi ); f_mul( &y, &p->Y, &zi );
  f_add( &a->ypx, &y, &x ); f_sub( &a->ymx, &y, &x ); f_mul( &a->xy2d, &x, &y ); f_mul( &a->xy2d, &a->xy2d, &F_D2 );
}

static void init( void ) {
  static const uint8_t d2[32] = { 0x59,0xf1,0xb2,0x26,0x94,0x9b,0xd6,0xeb,0x56,0xb1,0x83,0x82,0x9a,0x14,0xe0,0x00,
                                  0x30,0xd1,0xf3,0xee,0xf2,0x80,0x8e,0x19,0xe7,0xfc,0xdf,0x56,0xdc,0xd9,0x06,0x24 };
  static const uint8_t bx[32] = { 0x1a,0xd5,0x25,0x8f,0x60,0x2d,0x56,0xc9,0xb2,0xa7,0x25,0x95,0x60,0xc7,0x2c,0x69,
                                  0x5c,0xdc,0xd6,0xfd,0x31,0xe2,0xa4,0xc0,0xfe,0x53,0x6e,0xcd,0xd3,0x36,0x69,0x21 };
  uint8_t by[32]; memset( by, 0x66, 32 ); by[0] = 0x58;
  f_from( &F_D2, d2 );
  pt B; f_from( &B.X, bx ); f_from( &B.Y, by ); memset( &B.Z, 0, sizeof(f) ); B.Z.v[0] = 1; f_mul( &B.T, &B.X, &B.Y );
  pt base = B;
  for( int i=0; i<64; i++ ) {
    pt acc; pt_zero( &acc );
    for( int j=0; j<=8; j++ ) { to_aff( &comb[i][j], &acc ); pt_add( &acc, &acc, &base ); }
    for( int k=0; k<4; k++ ) pt_add( &base, &base, &base );   /* base *= 16 */
  }
}

/* [s]B, s 32 bytes LE with s < 2^255 */
static void smul_base( pt * r, uint8_t const s[32] ) {
  int8_t e[64]; int carry = 0;
  for( int i=0; i<63; i++ ) { int v = ((s[i>>1] >> (4*(i&1))) & 15) + carry; carry = (v+8)>>4; e[i] = (int8_t)(v - (carry<<4)); }
  e[63] = (int8_t)(((s[31] >> 4) & 7) + carry);   /* s < 2^255: top digit in [0,8], no carry out */
  pt_zero( r );
  for( int i=0; i<64; i++ ) { int d = e[i]; pt_madd( r, r, &comb[i][d<0?-d:d], d<0 ); }
}

/* ---- scalars mod l (schoolbook 512-bit, then Barrett-free bit reduction) -- */

static const uint64_t LW[4] = { 0x5812631a5cf5d3edUL, 0x14def9dea2f79cd6UL, 0, 0x1000000000000000UL };

static void sc_mod( uint8_t out[32], uint8_t const in[64] ) {
  /* r = in mod l by shift-subtract over 512 bits (test data generation only) */
  uint64_t r[5] = {0};
  for( int bit=511; bit>=0; bit-- ) {
    for( int i=4; i>0; i-- ) r[i] = r[i]<<1 | r[i-1]>>63;
    r[0] = r[0]<<1 | ((in[bit>>3] >> (bit&7)) & 1);
    /* if r >= l: r -= l */
    int ge = r[4] != 0;
    if( !ge ) { ge = 1; for( int i=3; i>=0; i-- ) { if( r[i] != LW[i] ) { ge = r[i] > LW[i]; break; } } }
    if( ge ) { u128 b = 0; for( int i=0; i<4; i++ ) { u128 d = (u128)r[i] - LW[i] - b; r[i] = (uint64_t)d; b = (d >> 64) & 1; } r[4] -= (uint64_t)b; }
  }
  for( int i=0; i<4; i++ ) for( int j=0; j<8; j++ ) out[8*i+j] = (uint8_t)(r[i] >> (8*j));
}
static void sc_muladd( uint8_t s[32], uint8_t const a[32], uint8_t const b[32], uint8_t const c[32] ) {
  uint64_t aw[4], bw[4], cw[4];
  for( int i=0; i<4; i++ ) { aw[i]=bw[i]=cw[i]=0; for( int j=7; j>=0; j-- ) { aw[i]=aw[i]<<8|a[8*i+j]; bw[i]=bw[i]<<8|b[8*i+j]; cw[i]=cw[i]<<8|c[8*i+j]; } }
  uint64_t w[8] = {0}; u128 carry = 0;
  for( int k=0; k<8; k++ ) {
    u128 lo = carry, hi = 0;
    for( int i=0; i<4; i++ ) { int j = k-i; if( j<0 || j>3 ) continue; u128 p = (u128)aw[i]*bw[j]; lo += (uint64_t)p; hi += (uint64_t)(p>>64); }
    if( k<4 ) lo += cw[k];
    w[k] = (uint64_t)lo; carry = (lo >> 64) + hi;
  }
  uint8_t wide[64]; for( int i=0; i<8; i++ ) for( int j=0; j<8; j++ ) wide[8*i+j] = (uint8_t)(w[i]>>(8*j));
  sc_mod( s, wide );
}

/* ---- keys and signing ------------------------------------------------------ */

typedef struct { uint8_t prv[32], pub[32], s[32], prefix[32]; } fdsynth_key_t;

void fdsynth_key( fdsynth_key_t * k, uint8_t const prv[32] ) {
  pthread_once( &once, init );
  uint8_t h[64]; sha_t sh; sha_init( &sh ); sha_add( &sh, prv, 32 ); sha_fin( &sh, h );
  h[0] &= 0xf8; h[31] &= 0x7f; h[31] |= 0x40;
  memcpy( k->prv, prv, 32 ); memcpy( k->s, h, 32 ); memcpy( k->prefix, h+32, 32 );
  pt A; smul_base( &A, k->s ); pt_enc( k->pub, &A );
}

void fdsynth_sign( uint8_t sig[64], uint8_t const * msg, size_t sz, fdsynth_key_t const * k ) {
  pthread_once( &once, init );
  uint8_t r[64], rr[32], h[64], kk[32]; sha_t sh;
  sha_init( &sh ); sha_add( &sh, k->prefix, 32 ); sha_add( &sh, msg, sz ); sha_fin( &sh, r );
  sc_mod( rr, r );
  pt R; smul_base( &R, rr ); pt_enc( sig, &R );
  sha_init( &sh ); sha_add( &sh, sig, 32 ); sha_add( &sh, k->pub, 32 ); sha_add( &sh, msg, sz ); sha_fin( &sh, h );
  sc_mod( kk, h );
  sc_muladd( sig+32, kk, k->s, rr );
}

/* ---- transactions ---------------------------------------------------------- */

static uint64_t xs( uint64_t * s ) { uint64_t x = *s; x ^= x<<13; x ^= x>>7; x ^= x<<17; *s = x; return x; }

#define FDSYNTH_LARGE_NOOP 0   /* 1232-byte single signer (fd_benchg large_noop_t) */
#define FDSYNTH_SMALL_MSG  1   /* single signer, 200-byte message (BASELINE config 0) */
#define FDSYNTH_MULTI      2   /* n signers (1..max_signers), shared message, <=1232 bytes */

/* Expected codes of the injected faults under AVX-512 semantics
   (SURVEY.md §8d C3): S>=l, undecodable R, undecodable A, small-order R,
   small-order A, 1-bit message flip. */
static const int8_t fault_code[6] = { -1, -1, -1, -1, -2, -3 };

typedef struct {
  uint8_t * payload; fdgpu_txn_desc_t * desc; int8_t * expect;
  fdsynth_key_t const * keys; size_t nkeys;
  size_t lo, hi, stride; int kind, max_signers; double invalid; uint64_t seed;
} job_t;

static size_t txn_layout( int kind, int nsig, size_t * msg_off ) {
  if( kind==FDSYNTH_SMALL_MSG ) { *msg_off = 65; return 65 + 200; }
  *msg_off = 1 + 64*(size_t)nsig;
  return 1232;
}

static void * job( void * _j ) {
  job_t * j = (job_t *)_j;
  uint8_t const l_le[32] = { 0xed,0xd3,0xf5,0x5c,0x1a,0x63,0x12,0x58,0xd6,0x9c,0xf7,0xa2,0xde,0xf9,0xde,0x14,
                             0,0,0,0,0,0,0,0,0,0,0,0,0,0,0,0x10 };
  for( size_t t=j->lo; t<j->hi; t++ ) {
    uint64_t st = j->seed ^ (0x9e3779b97f4a7c15UL * (t+1)); xs( &st ); xs( &st );
    int nsig = 1;
    if( j->kind==FDSYNTH_MULTI ) nsig = 1 + (int)(xs( &st ) % (uint64_t)j->max_signers);
    size_t msg_off; size_t sz = txn_layout( j->kind, nsig, &msg_off );
    uint8_t * p = j->payload + t * j->stride;
    fdgpu_txn_desc_t * d = j->desc + t;
    /* body: a well-formed legacy message (fd_txn_parse accepts it):
       header, accounts (signers first, then the program ids),
       blockhash, instructions.  LARGE_NOOP / SMALL_MSG follow fd_benchg's
       large_noop_t (fd_benchg.c:102-171): 3 accounts, a 9-byte compute
       budget instruction and a filler instruction to the program at
       account 2; MULTI has nsig+1 accounts and one filler instruction
       (which is what lets 12 signers fit in 1232 bytes). */
    uint8_t * m = p + msg_off;
    size_t msz = sz - msg_off;
    for( size_t i=0; i<msz; i+=8 ) { uint64_t x = xs( &st ); size_t n = msz-i < 8 ? msz-i : 8; memcpy( m+i, &x, n ); }
    int nprog = j->kind==FDSYNTH_MULTI ? 1 : 2;
    size_t acct = (size_t)nsig + (size_t)nprog;
    p[0] = (uint8_t)nsig;
    m[0] = (uint8_t)nsig; m[1] = 0; m[2] = (uint8_t)nprog; m[3] = (uint8_t)acct;
    {
      uint8_t * q = m + 4 + 32*acct + 32;             /* after accounts and blockhash */
      *q++ = (uint8_t)nprog;                           /* instr_cnt */
      if( nprog==2 ) { q[0] = (uint8_t)nsig; q[1] = 0; q[2] = 9; q[3] = 3; q += 12; }   /* set CU price */
      size_t rem = (size_t)( (m + msz) - q ) - 2;      /* prog_id + acct_cnt */
      size_t dsz = rem - 1 <= 127 ? rem - 1 : rem - 2; /* compact-u16 data_sz (sizes here never hit 129) */
      q[0] = (uint8_t)( nsig + nprog - 1 ); q[1] = 0; q += 2;
      if( dsz <= 127 ) *q++ = (uint8_t)dsz;
      else { *q++ = (uint8_t)( 0x80 | (dsz & 0x7f) ); *q++ = (uint8_t)( dsz >> 7 ); }
    }
    fdsynth_key_t const * ks[16];
    for( int s=0; s<nsig; s++ ) { ks[s] = &j->keys[ (t*7 + (size_t)s*13 + (xs( &st ) & 3)) % j->nkeys ]; memcpy( m + 4 + 32*s, ks[s]->pub, 32 ); }
    int8_t code = 0;
    int fault = -1, fj = 0;
    if( j->invalid > 0 && (double)(xs( &st ) >> 11) * (1.0/9007199254740992.0) < j->invalid ) {
      fault = (int)(xs( &st ) % 6); fj = (int)(xs( &st ) % (uint64_t)nsig); code = fault_code[fault];
    }
    if( fault==2 || fault==4 ) {   /* replace signer fj's pubkey in the message before signing */
      uint8_t * a = m + 4 + 32*fj; memset( a, 0, 32 );
      a[0] = fault==2 ? 2 : 1;       /* y=2: not on the curve; y=1: identity (small order) */
    }
    for( int s=0; s<nsig; s++ ) fdsynth_sign( p + 1 + 64*s, m, msz, ks[s] );
    if( fault==0 ) { /* S += l */
      uint8_t * S = p + 1 + 64*fj + 32; unsigned c = 0;
      for( int i=0; i<32; i++ ) { c += (unsigned)S[i] + l_le[i]; S[i] = (uint8_t)c; c >>= 8; }
    } else if( fault==1 ) { uint8_t * R = p + 1 + 64*fj; memset( R, 0, 32 ); R[0] = 2; }
    else if( fault==3 ) { uint8_t * R = p + 1 + 64*fj; memset( R, 0, 32 ); R[0] = 1; }
    else if( fault==5 ) { m[msz-1] ^= 0x01; }
    d->payload_off = (unsigned)(t * j->stride); d->payload_sz = (unsigned short)sz;
    d->signature_off = 1; d->message_off = (unsigned short)msg_off; d->acct_addr_off = (unsigned short)(msg_off + 4);
    d->sig_cnt = (unsigned char)nsig; d->sig_base = 0;
    if( j->expect ) j->expect[t] = code;
  }
  return NULL;
}

void fdsynth_keys( fdsynth_key_t * keys, size_t n, uint64_t seed ) {
  uint64_t st = seed | 1;
  for( size_t i=0; i<n; i++ ) {
    uint8_t prv[32]; for( int k=0; k<4; k++ ) { uint64_t x = xs( &st ); memcpy( prv + 8*k, &x, 8 ); }
    fdsynth_key( keys + i, prv );
  }
}

/* Generate n transactions at payload + t*stride (stride >= 1232, a
   multiple of 8), fill desc (sig_base prefix included) and the intended
   per-txn code under AVX-512 semantics.  Returns the signature count. */
size_t fdsynth_txns( uint8_t * payload, size_t stride, fdgpu_txn_desc_t * desc, int8_t * expect, size_t n,
                     int kind, int max_signers, double invalid_frac, uint64_t seed,
                     fdsynth_key_t const * keys, size_t nkeys, int threads ) {
  pthread_once( &once, init );
  if( threads < 1 ) threads = 1;
  if( threads > 64 ) threads = 64;
  if( max_signers < 1 ) max_signers = 1;
  if( max_signers > 12 ) max_signers = 12;   /* 13 signer accounts no longer fit 1232 bytes */
  pthread_t th[64]; job_t jb[64];
  for( int i=0; i<threads; i++ ) {
    jb[i] = (job_t){ payload, desc, expect, keys, nkeys, n*(size_t)i/(size_t)threads, n*(size_t)(i+1)/(size_t)threads,
                     stride, kind, max_signers, invalid_frac, seed };
    if( i ) pthread_create( &th[i], NULL, job, &jb[i] );
  }
  job( &jb[0] );
  for( int i=1; i<threads; i++ ) pthread_join( th[i], NULL );
  size_t s = 0;
  for( size_t t=0; t<n; t++ ) { desc[t].sig_base = (unsigned)s; s += desc[t].sig_cnt; }
  return s;
}
