/* fd_txn_oracle.c -- TEST INFRASTRUCTURE ONLY.

   From-scratch CPU restatement of the Solana transaction parser the
   verify tile runs before signature verification (after_frag,
   src/disco/verify/fd_verify_tile.c:110-113):

     fd_txn_parse / fd_txn_parse_core  src/ballet/txn/fd_txn_parse.c:6-252
     compact-u16 decoding              src/ballet/txn/fd_compact_u16.h:34-87
     fd_txn_t layout and footprint     src/ballet/txn/fd_txn.h:139-352, :481-487

   It is the checker for the device parser (fd_txn_parse_gpu.h) and is
   itself pinned against the reference parser compiled in place
   (oracle/_ref/libfdref_txn.so) on the reference's own fixtures
   (src/ballet/txn/fixtures/transaction{1..6}.bin) and on the mutation
   sweep of src/ballet/txn/test_txn_parse.c:137-220 (tests/golden/txn_parse.npz).

   Output: the fd_txn_t image (little-endian, the reference's packed
   field order, written into out[0..footprint) and the footprint, or 0
   when the payload is rejected.  On rejection the contents of out are
   unspecified (the reference also leaves a partial image). */

#include <stdint.h>
#include <string.h>

#define TXN_MTU          1232u   /* FD_TXN_MTU            fd_txn.h:104 */
#define TXN_SIG_MAX       127u   /* FD_TXN_SIG_MAX        fd_txn.h:67  */
#define TXN_ACCT_MAX      128u   /* FD_TXN_ACCT_ADDR_MAX  fd_txn.h:77  */
#define TXN_LUT_MAX       127u   /* FD_TXN_ADDR_TABLE_LOOKUP_MAX :86   */
#define TXN_INSTR_MAX      64u   /* FD_TXN_INSTR_MAX      fd_txn.h:90  */
#define TXN_HDR_SZ         20u   /* sizeof(fd_txn_t)                   */
#define TXN_INSTR_SZ       10u   /* sizeof(fd_txn_instr_t)             */
#define TXN_LUT_SZ          8u   /* sizeof(fd_txn_acct_addr_lut_t)     */
#define TXN_V0           0x00u
#define TXN_VLEGACY      0xffu

typedef struct {
  uint8_t const * p;
  uint32_t        sz;
  uint32_t        i;     /* bytes consumed; invariant i <= sz */
} cur_t;

/* bytes left >= n (n is attacker controlled: compare without i+n) */
static int have( cur_t const * c, uint32_t n ) { return n <= c->sz - c->i; }

/* compact-u16 (minimal encoding, value < 2^16); returns its width 1..3 or 0 */
static uint32_t
cu16( cur_t const * c, uint32_t * val ) {
  uint32_t left = c->sz - c->i;
  uint8_t const * b = c->p + c->i;
  if( left >= 1u && b[0] < 0x80u ) { *val = b[0]; return 1u; }
  if( left >= 2u && b[1] < 0x80u ) {
    if( b[1]==0u ) return 0u;                               /* non-minimal */
    *val = (uint32_t)(b[0] & 0x7fu) | ((uint32_t)b[1] << 7);
    return 2u;
  }
  if( left >= 3u && b[2] < 0x04u ) {
    if( b[2]==0u ) return 0u;                               /* non-minimal */
    *val = (uint32_t)(b[0] & 0x7fu) | ((uint32_t)(b[1] & 0x7fu) << 7) | ((uint32_t)b[2] << 14);
    return 3u;
  }
  return 0u;
}

static void put8 ( uint8_t * o, uint32_t off, uint32_t v ) { o[off] = (uint8_t)v; }
static void put16( uint8_t * o, uint32_t off, uint32_t v ) { o[off] = (uint8_t)v; o[off+1] = (uint8_t)(v >> 8); }

#define NEED( n )   do { if( !have( &c, (n) ) ) return 0u; } while(0)
#define REQ( cond ) do { if( !(cond) ) return 0u; } while(0)
#define CU16( v )   do { uint32_t _w = cu16( &c, &(v) ); REQ( _w ); c.i += _w; } while(0)

uint32_t
oracle_txn_parse( uint8_t const * payload, uint32_t payload_sz, uint8_t * out ) {
  REQ( payload_sz <= TXN_MTU );
  cur_t c = { payload, payload_sz, 0u };

  NEED( 1u ); uint32_t sig_cnt = payload[ c.i++ ];
  REQ( sig_cnt >= 1u && sig_cnt <= TXN_SIG_MAX );
  NEED( 64u*sig_cnt ); uint32_t sig_off = c.i; c.i += 64u*sig_cnt;

  uint32_t msg_off = c.i;
  NEED( 1u ); uint32_t b0 = payload[ c.i++ ];
  uint32_t ver;
  if( b0 & 0x80u ) {                                  /* versioned message */
    ver = b0 & 0x7fu;
    REQ( ver==TXN_V0 );
    NEED( 1u ); REQ( payload[ c.i ]==sig_cnt ); c.i++;
  } else {
    ver = TXN_VLEGACY;
    REQ( b0==sig_cnt );
  }
  NEED( 1u ); uint32_t ro_signed   = payload[ c.i++ ];
  REQ( ro_signed < sig_cnt );
  NEED( 1u ); uint32_t ro_unsigned = payload[ c.i++ ];

  uint32_t acct_cnt; CU16( acct_cnt );
  REQ( sig_cnt <= acct_cnt && acct_cnt <= TXN_ACCT_MAX );
  REQ( sig_cnt + ro_unsigned <= acct_cnt );
  NEED( 32u*acct_cnt ); uint32_t acct_off = c.i; c.i += 32u*acct_cnt;
  NEED( 32u );          uint32_t bh_off   = c.i; c.i += 32u;

  uint32_t instr_cnt; CU16( instr_cnt );
  REQ( instr_cnt <= TXN_INSTR_MAX );
  NEED( 3u*instr_cnt );                              /* 3 B = smallest instruction */
  REQ( acct_cnt > (instr_cnt ? 1u : 0u) );

  put8 ( out,  0, ver );        put8 ( out,  1, sig_cnt );
  put16( out,  2, sig_off );    put16( out,  4, msg_off );
  put8 ( out,  6, ro_signed );  put8 ( out,  7, ro_unsigned );
  put16( out,  8, acct_cnt );   put16( out, 10, acct_off );
  put16( out, 12, bh_off );     put16( out, 18, instr_cnt );

  uint32_t max_acct = 0u;
  for( uint32_t j=0u; j<instr_cnt; j++ ) {
    NEED( 3u ); uint32_t prog = payload[ c.i++ ];
    uint32_t n_acct; CU16( n_acct );
    NEED( n_acct ); uint32_t a_off = c.i;
    for( uint32_t k=0u; k<n_acct; k++ ) if( payload[ a_off+k ] > max_acct ) max_acct = payload[ a_off+k ];
    c.i += n_acct;
    uint32_t d_sz; CU16( d_sz );
    NEED( d_sz ); uint32_t d_off = c.i; c.i += d_sz;
    REQ( prog > 0u && prog < acct_cnt );               /* not the fee payer, in range */
    uint8_t * ix = out + TXN_HDR_SZ + TXN_INSTR_SZ*j;
    put8( ix, 0, prog ); put8( ix, 1, 0u ); put16( ix, 2, n_acct ); put16( ix, 4, d_sz );
    put16( ix, 6, a_off ); put16( ix, 8, d_off );
  }

  uint32_t lut_cnt = 0u, adtl_w = 0u, adtl = 0u;
  if( ver==TXN_V0 ) {
    CU16( lut_cnt );
    REQ( lut_cnt <= TXN_LUT_MAX );
    NEED( 34u*lut_cnt );                              /* 32 B key + two 1-B counts */
    uint8_t * lut = out + TXN_HDR_SZ + TXN_INSTR_SZ*instr_cnt;
    for( uint32_t j=0u; j<lut_cnt; j++ ) {
      NEED( 32u ); uint32_t k_off = c.i; c.i += 32u;
      uint32_t nw; CU16( nw );
      NEED( nw ); uint32_t w_off = c.i; c.i += nw;
      uint32_t nr; CU16( nr );
      NEED( nr ); uint32_t r_off = c.i; c.i += nr;
      REQ( nw <= TXN_ACCT_MAX - acct_cnt );
      REQ( nr <= TXN_ACCT_MAX - acct_cnt );
      REQ( nw + nr >= 1u );
      uint8_t * e = lut + TXN_LUT_SZ*j;
      put16( e, 0, k_off ); put8( e, 2, nw ); put8( e, 3, nr ); put16( e, 4, w_off ); put16( e, 6, r_off );
      adtl_w += nw; adtl += nw + nr;
    }
  }
  REQ( c.i==payload_sz );                             /* no trailing bytes */
  REQ( acct_cnt + adtl <= TXN_ACCT_MAX );
  REQ( max_acct < acct_cnt + adtl );

  put8( out, 14, lut_cnt ); put8( out, 15, adtl_w ); put8( out, 16, adtl ); put8( out, 17, 0u );
  return TXN_HDR_SZ + TXN_INSTR_SZ*instr_cnt + TXN_LUT_SZ*lut_cnt;
}

/* batch form: payloads at arena + off[t], sizes sz[t]; images at
   out + t*stride; footprints (0 = rejected) to fp[t] */
void
oracle_txn_parse_batch( uint8_t const * arena, uint32_t const * off, uint16_t const * sz, uint64_t n,
                        uint8_t * out, uint64_t stride, uint16_t * fp ) {
  for( uint64_t t=0; t<n; t++ ) fp[t] = (uint16_t)oracle_txn_parse( arena + off[t], sz[t], out + t*stride );
}
