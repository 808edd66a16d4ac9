#pragma once
/* fd_gpu_txn.h -- Solana transaction parser, one transaction per lane
   (CDNA4 device code).

   Device-side replacement for the fd_txn_parse call the verify tile makes
   before verification (src/disco/verify/fd_verify_tile.c:110-113):
   fd_txn_parse_core (src/ballet/txn/fd_txn_parse.c:6-252) with the
   compact-u16 rules of src/ballet/txn/fd_compact_u16.h:34-87, producing
   the same fd_txn_t image (src/ballet/txn/fd_txn.h:139-352) and the same
   footprint (fd_txn.h:481-487), 0 on rejection.

   The payload is walked with byte loads; every read is preceded by a
   bound check against the remaining length (n <= sz - i, never i + n),
   so a hostile payload cannot make a lane read outside [0, sz).  The
   image is written with byte / halfword stores into the lane's own
   slot; on rejection the slot holds a partial image (as in the
   reference) and the footprint says 0. */

#include <hip/hip_runtime.h>
#include <stdint.h>

#define FDGPU_TXN_IMG_HDR   20u    /* sizeof(fd_txn_t)                */
#define FDGPU_TXN_IMG_INSTR 10u    /* sizeof(fd_txn_instr_t)          */
#define FDGPU_TXN_IMG_LUT    8u    /* sizeof(fd_txn_acct_addr_lut_t)  */

struct fd_txn_cur {
  unsigned char const * p;
  uint32_t              sz;
  uint32_t              i;
};

__device__ __forceinline__ int fd_txn_have( fd_txn_cur const & c, uint32_t n ) { return n <= c.sz - c.i; }

/* compact-u16 at the cursor: width 1..3, or 0 if truncated / non-minimal / > 16 bits */
__device__ __forceinline__ uint32_t
fd_txn_cu16( fd_txn_cur const & c, uint32_t & v ) {
  uint32_t left = c.sz - c.i;
  if( left == 0u ) return 0u;
  uint32_t b0 = c.p[ c.i ];
  if( b0 < 0x80u ) { v = b0; return 1u; }
  if( left == 1u ) return 0u;
  uint32_t b1 = c.p[ c.i + 1u ];
  if( b1 < 0x80u ) {
    if( b1 == 0u ) return 0u;
    v = (b0 & 0x7fu) | (b1 << 7);
    return 2u;
  }
  if( left == 2u ) return 0u;
  uint32_t b2 = c.p[ c.i + 2u ];
  if( b2 >= 0x04u || b2 == 0u ) return 0u;
  v = (b0 & 0x7fu) | ((b1 & 0x7fu) << 7) | (b2 << 14);
  return 3u;
}

__device__ __forceinline__ void fd_img8 ( unsigned char * o, uint32_t off, uint32_t v ) { o[off] = (unsigned char)v; }
__device__ __forceinline__ void fd_img16( unsigned char * o, uint32_t off, uint32_t v ) {
  o[off] = (unsigned char)v; o[off+1u] = (unsigned char)(v >> 8);
}

/* header fields the verify path needs, valid when the return is nonzero */
struct fd_txn_hdr {
  uint32_t sig_cnt, sig_off, msg_off, acct_off;
};

#define FD_TXN_NEED( n )   do { if( !fd_txn_have( c, (n) ) ) return 0u; } while(0)
#define FD_TXN_REQ( cond ) do { if( !(cond) ) return 0u; } while(0)
#define FD_TXN_CU16( v )   do { uint32_t _w = fd_txn_cu16( c, (v) ); FD_TXN_REQ( _w ); c.i += _w; } while(0)

/* Parse payload[0,sz) into img (may be NULL: header only).  Returns the
   fd_txn_t footprint or 0. */
__device__ uint32_t
fd_txn_parse_dev( unsigned char const * payload, uint32_t sz, unsigned char * img, fd_txn_hdr & h ) {
  FD_TXN_REQ( sz <= 1232u );                                   /* FD_TXN_MTU */
  fd_txn_cur c = { payload, sz, 0u };

  FD_TXN_NEED( 1u ); uint32_t sig_cnt = payload[ c.i++ ];
  FD_TXN_REQ( sig_cnt >= 1u && sig_cnt <= 127u );              /* FD_TXN_SIG_MAX */
  FD_TXN_NEED( 64u*sig_cnt ); uint32_t sig_off = c.i; c.i += 64u*sig_cnt;
  uint32_t msg_off = c.i;
  FD_TXN_NEED( 1u ); uint32_t b0 = payload[ c.i++ ];
  uint32_t ver;
  if( b0 & 0x80u ) {
    ver = b0 & 0x7fu;
    FD_TXN_REQ( ver == 0u );                                   /* only v0 is defined */
    FD_TXN_NEED( 1u ); FD_TXN_REQ( payload[ c.i ] == sig_cnt ); c.i++;
  } else {
    ver = 0xffu;                                               /* legacy */
    FD_TXN_REQ( b0 == sig_cnt );
  }
  FD_TXN_NEED( 1u ); uint32_t ro_signed   = payload[ c.i++ ];
  FD_TXN_REQ( ro_signed < sig_cnt );
  FD_TXN_NEED( 1u ); uint32_t ro_unsigned = payload[ c.i++ ];
  uint32_t acct_cnt; FD_TXN_CU16( acct_cnt );
  FD_TXN_REQ( sig_cnt <= acct_cnt && acct_cnt <= 128u );       /* FD_TXN_ACCT_ADDR_MAX */
  FD_TXN_REQ( sig_cnt + ro_unsigned <= acct_cnt );
  FD_TXN_NEED( 32u*acct_cnt ); uint32_t acct_off = c.i; c.i += 32u*acct_cnt;
  FD_TXN_NEED( 32u );          uint32_t bh_off   = c.i; c.i += 32u;
  uint32_t instr_cnt; FD_TXN_CU16( instr_cnt );
  FD_TXN_REQ( instr_cnt <= 64u );                              /* FD_TXN_INSTR_MAX */
  FD_TXN_NEED( 3u*instr_cnt );
  FD_TXN_REQ( acct_cnt > ( instr_cnt ? 1u : 0u ) );

  if( img ) {
    fd_img8 ( img,  0, ver );       fd_img8 ( img,  1, sig_cnt );
    fd_img16( img,  2, sig_off );   fd_img16( img,  4, msg_off );
    fd_img8 ( img,  6, ro_signed ); fd_img8 ( img,  7, ro_unsigned );
    fd_img16( img,  8, acct_cnt );  fd_img16( img, 10, acct_off );
    fd_img16( img, 12, bh_off );    fd_img16( img, 18, instr_cnt );
  }

  uint32_t max_acct = 0u;
  for( uint32_t j=0u; j<instr_cnt; j++ ) {
    FD_TXN_NEED( 3u ); uint32_t prog = payload[ c.i++ ];
    uint32_t n_acct; FD_TXN_CU16( n_acct );
    FD_TXN_NEED( n_acct ); uint32_t a_off = c.i;
    for( uint32_t k=0u; k<n_acct; k++ ) max_acct = max( max_acct, (uint32_t)payload[ a_off + k ] );
    c.i += n_acct;
    uint32_t d_sz; FD_TXN_CU16( d_sz );
    FD_TXN_NEED( d_sz ); uint32_t d_off = c.i; c.i += d_sz;
    FD_TXN_REQ( prog > 0u && prog < acct_cnt );
    if( img ) {
      unsigned char * ix = img + FDGPU_TXN_IMG_HDR + FDGPU_TXN_IMG_INSTR*j;
      fd_img8( ix, 0, prog ); fd_img8( ix, 1, 0u ); fd_img16( ix, 2, n_acct ); fd_img16( ix, 4, d_sz );
      fd_img16( ix, 6, a_off ); fd_img16( ix, 8, d_off );
    }
  }

  uint32_t lut_cnt = 0u, adtl_w = 0u, adtl = 0u;
  if( ver == 0u ) {
    FD_TXN_CU16( lut_cnt );
    FD_TXN_REQ( lut_cnt <= 127u );                             /* FD_TXN_ADDR_TABLE_LOOKUP_MAX */
    FD_TXN_NEED( 34u*lut_cnt );
    for( uint32_t j=0u; j<lut_cnt; j++ ) {
      FD_TXN_NEED( 32u ); uint32_t k_off = c.i; c.i += 32u;
      uint32_t nw; FD_TXN_CU16( nw );
      FD_TXN_NEED( nw ); uint32_t w_off = c.i; c.i += nw;
      uint32_t nr; FD_TXN_CU16( nr );
      FD_TXN_NEED( nr ); uint32_t r_off = c.i; c.i += nr;
      FD_TXN_REQ( nw <= 128u - acct_cnt );
      FD_TXN_REQ( nr <= 128u - acct_cnt );
      FD_TXN_REQ( nw + nr >= 1u );
      if( img ) {
        unsigned char * e = img + FDGPU_TXN_IMG_HDR + FDGPU_TXN_IMG_INSTR*instr_cnt + FDGPU_TXN_IMG_LUT*j;
        fd_img16( e, 0, k_off ); fd_img8( e, 2, nw ); fd_img8( e, 3, nr ); fd_img16( e, 4, w_off ); fd_img16( e, 6, r_off );
      }
      adtl_w += nw; adtl += nw + nr;
    }
  }
  FD_TXN_REQ( c.i == sz );
  FD_TXN_REQ( acct_cnt + adtl <= 128u );
  FD_TXN_REQ( max_acct < acct_cnt + adtl );
  if( img ) { fd_img8( img, 14, lut_cnt ); fd_img8( img, 15, adtl_w ); fd_img8( img, 16, adtl ); fd_img8( img, 17, 0u ); }
  h.sig_cnt = sig_cnt; h.sig_off = sig_off; h.msg_off = msg_off; h.acct_off = acct_off;
  return FDGPU_TXN_IMG_HDR + FDGPU_TXN_IMG_INSTR*instr_cnt + FDGPU_TXN_IMG_LUT*lut_cnt;
}

#undef FD_TXN_NEED
#undef FD_TXN_REQ
#undef FD_TXN_CU16
