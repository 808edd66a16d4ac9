/* ref_tile_harness.c -- TEST INFRASTRUCTURE ONLY.

   The reference verify tile's per-frag decision, built from the
   reference's own code compiled in place from /root/reference by
   oracle/Makefile (never copied): fd_txn_verify and fd_verify_ctx_t
   (src/disco/verify/fd_verify_tile.h:17-108, header-inline), the
   FD_TCACHE_QUERY / FD_TCACHE_INSERT macros and fd_tcache_remove
   (src/tango/tcache/fd_tcache.h:281-404), fd_hash (src/util/fd_hash.c),
   fd_txn_parse (src/ballet/txn/fd_txn_parse.c), the fd_txn_m_t helpers
   (src/disco/fd_txn_m_t.h) and fd_ed25519_verify_batch_single_msg with
   its AVX-512 backend.  The only code here is the loop over frags and
   the tile's frag callbacks, restated statement for statement from
   src/disco/verify/fd_verify_tile.c: before_frag (:36-59), during_frag
   (:65-101) and after_frag's bundle bookkeeping (:103-157) -- static
   functions of the tile's translation unit, which needs the stem and
   topo runtime.  The gossip update message is the reference's own
   fd_gossip_update_message_t (src/flamenco/gossip/fd_gossip_types.h,
   compiled in place).  libfdref_tile.so is the expectation of
   tests/test_gpu_vtile.py: every frag's outcome, the four metrics and the
   published fd_txn_m_t records. */

#include <limits.h>
#include <stdlib.h>
#include <string.h>
#include "disco/verify/fd_verify_tile.h"
#include "disco/fd_txn_m_t.h"
#include "ballet/txn/fd_txn.h"
#include "ballet/ed25519/fd_ed25519.h"
#include "flamenco/gossip/fd_gossip_types.h"

/* outcomes, as include/fd_verify_gpu.h's FDGPU_VTILE_* */
#define R_PUBLISH 0
#define R_PARSE   1
#define R_VERIFY  2
#define R_DEDUP   3
#define R_PEER    4
#define R_SKIP   -2        /* before_frag filtered it out (this tile never sees it) */

/* in kinds, fd_verify_tile.c:7-10 */
#define K_QUIC   0UL
#define K_BUNDLE 1UL
#define K_GOSSIP 2UL
#define K_SEND   3UL

typedef struct {
  fd_verify_ctx_t * ctx;
  ulong *           ring;
  ulong *           map;
  ulong             oldest;
  fd_sha512_t *     sha;
  uchar *           buf;         /* the out dcache chunk the tile writes into (reused until a publish) */
} ref_tile_t;

static int
ref_tile_init( ref_tile_t * t, ulong depth, ulong seed, ulong rec_stride ) {
  memset( t, 0, sizeof(*t) );
  t->ctx = (fd_verify_ctx_t *)calloc( 1, sizeof(fd_verify_ctx_t) );
  t->sha = (fd_sha512_t *)aligned_alloc( FD_SHA512_ALIGN, FD_TXN_ACTUAL_SIG_MAX * sizeof(fd_sha512_t) );
  ulong map_cnt = fd_tcache_map_cnt_default( depth );
  t->ring = (ulong *)malloc( depth * sizeof(ulong) );
  t->map  = (ulong *)malloc( map_cnt * sizeof(ulong) );
  t->buf  = (uchar *)aligned_alloc( 64, rec_stride );
  if( !t->ctx || !t->sha || !t->ring || !t->map || !t->buf || !map_cnt ) return -1;
  memset( t->buf, 0, rec_stride );
  fd_verify_ctx_t * ctx = t->ctx;
  for( ulong i=0UL; i<FD_TXN_ACTUAL_SIG_MAX; i++ ) ctx->sha[i] = fd_sha512_init( t->sha + i );
  t->oldest = fd_tcache_reset( t->ring, depth, t->map, map_cnt );
  ctx->tcache_depth = depth; ctx->tcache_map_cnt = map_cnt;
  ctx->tcache_sync = &t->oldest; ctx->tcache_ring = t->ring; ctx->tcache_map = t->map;
  ctx->hashmap_seed = seed;
  return 0;
}

static void
ref_tile_fini( ref_tile_t * t ) {
  free( t->ctx ); free( t->sha ); free( t->ring ); free( t->map ); free( t->buf );
}

/* after_frag, fd_verify_tile.c:114-156, on the record in t->buf: the outcome; a published record's
   realized size in *rec_sz and its HA dedup tag in *tag */
static int
ref_after_frag( ref_tile_t * t, ulong * rec_sz, ulong * tag ) {
  fd_verify_ctx_t * ctx = t->ctx;
  fd_txn_m_t * txnm = (fd_txn_m_t *)t->buf;
  fd_txn_t * txnt = fd_txn_m_txn_t( txnm );
  txnm->txn_t_sz = (ushort)fd_txn_parse( fd_txn_m_payload( txnm ), txnm->payload_sz, txnt, NULL );
  int is_bundle = !!txnm->block_engine.bundle_id;
  if( is_bundle & (txnm->block_engine.bundle_id!=ctx->bundle_id) ) {
    ctx->bundle_failed = 0;
    ctx->bundle_id     = txnm->block_engine.bundle_id;
  }
  if( is_bundle & (!!ctx->bundle_failed) ) { ctx->metrics.bundle_peer_fail_cnt++; return R_PEER; }
  if( !txnm->txn_t_sz ) {
    if( is_bundle ) ctx->bundle_failed = 1;
    ctx->metrics.parse_fail_cnt++; return R_PARSE;
  }
  ulong txn_sig = 0UL;
  int r = fd_txn_verify( ctx, fd_txn_m_payload( txnm ), txnm->payload_sz, txnt, !is_bundle, &txn_sig );
  if( r!=FD_TXN_VERIFY_SUCCESS ) {
    if( is_bundle ) ctx->bundle_failed = 1;
    if( r==FD_TXN_VERIFY_DEDUP ) { ctx->metrics.dedup_fail_cnt++; return R_DEDUP; }
    ctx->metrics.verify_fail_cnt++; return R_VERIFY;
  }
  *rec_sz = fd_txn_m_realized_footprint( txnm, 1, 0 );
  *tag = is_bundle ? 0UL : txn_sig;
  return R_PUBLISH;
}

/* before_frag, fd_verify_tile.c:36-59: 1 = skip */
static int
ref_before_frag( ulong rr_idx, ulong rr_cnt, ulong in_kind, ulong seq, ulong sig ) {
  int is_bundle_packet = (in_kind==K_BUNDLE && !sig);
  if( is_bundle_packet || in_kind==K_QUIC ) return (seq % rr_cnt) != rr_idx;
  else if( in_kind==K_BUNDLE ) return rr_idx!=0UL;
  else if( in_kind==K_GOSSIP ) return (seq % rr_cnt) != rr_idx || sig!=FD_GOSSIP_UPDATE_TAG_VOTE;
  return 0;
}

/* during_frag, fd_verify_tile.c:65-101 (the range checks that FD_LOG_ERR are the caller's: it only
   passes well-formed frags): the frag's bytes land in the out chunk t->buf */
static void
ref_during_frag( ref_tile_t * t, ulong in_kind, uchar const * src, ulong sz ) {
  if( in_kind==K_BUNDLE || in_kind==K_QUIC || in_kind==K_SEND ) {
    memcpy( t->buf, src, sz );
  } else if( in_kind==K_GOSSIP ) {
    fd_gossip_update_message_t const * msg = (fd_gossip_update_message_t const *)src;
    fd_txn_m_t * dst = (fd_txn_m_t *)t->buf;
    dst->payload_sz = (ushort)msg->vote.txn_sz;
    dst->block_engine.bundle_id = 0UL;
    memcpy( fd_txn_m_payload( dst ), msg->vote.txn, msg->vote.txn_sz );
  }
}

/* The full frag path of one tile (verify:rr_idx of rr_cnt) over a mixed stream: frag i of in kind kind[i]
   with stem seq seq[i] and mcache sig sig[i] is arena[off[i], off[i]+sz[i]) -- an fd_txn_m_t record
   (header + payload) for QUIC / bundle / send frags, an fd_gossip_update_message_t for gossip frags.
   res[i] = R_SKIP when before_frag filters it, else the after_frag outcome; published records and tags
   as ref_tile_run.  0, or -1. */
int
ref_tile_run_kinds( uchar const * arena, uint const * off, ushort const * sz, ulong const * kind, ulong const * seq,
                    ulong const * sig, ulong n, ulong rr_idx, ulong rr_cnt, ulong depth, ulong seed, int * res,
                    ulong * rec_sz, uchar * rec, ulong rec_stride, ulong * tag, ulong metrics[ 5 ] ) {
  if( !depth || !rr_cnt || rr_idx >= rr_cnt || rec_stride < FD_TPU_MTU + 1024UL ) return -1;
  ref_tile_t t;
  if( ref_tile_init( &t, depth, seed, rec_stride ) ) { ref_tile_fini( &t ); return -1; }
  memset( metrics, 0, 5UL*sizeof(ulong) );
  for( ulong i=0UL; i<n; i++ ) {
    res[i] = R_SKIP; rec_sz[i] = 0UL; tag[i] = 0UL;
    if( ref_before_frag( rr_idx, rr_cnt, kind[i], seq[i], sig[i] ) ) continue;
    ref_during_frag( &t, kind[i], arena + off[i], sz[i] );
    res[i] = ref_after_frag( &t, rec_sz + i, tag + i );
    if( res[i]==R_PUBLISH ) { memcpy( rec + i*rec_stride, t.buf, rec_sz[i] ); metrics[4]++; }
  }
  metrics[0] = t.ctx->metrics.parse_fail_cnt; metrics[1] = t.ctx->metrics.verify_fail_cnt;
  metrics[2] = t.ctx->metrics.dedup_fail_cnt; metrics[3] = t.ctx->metrics.bundle_peer_fail_cnt;
  ref_tile_fini( &t );
  return 0;
}

/* frag i: payload arena[off[i], off[i]+sz[i]), bundle id bid[i].  Out:
   res[i]; for published frags rec_sz[i] = fd_txn_m_realized_footprint and
   the record (fd_txn_m_t header + payload + fd_txn_t) in rec + i*rec_stride;
   tag[i] = the HA dedup tag fd_txn_verify returned (0 for bundles, as the
   stem publishes sig 0); metrics: parse, verify, dedup, bundle peer,
   published.  Returns 0, or -1 on a bad argument. */
int
ref_tile_run( uchar const * arena, uint const * off, ushort const * sz, ulong const * bid, ulong n,
              ulong depth, ulong seed, int * res, ulong * rec_sz, uchar * rec, ulong rec_stride, ulong * tag,
              ulong metrics[ 5 ] ) {
  if( !depth || rec_stride < FD_TPU_MTU + 1024UL ) return -1;
  ref_tile_t t;
  if( ref_tile_init( &t, depth, seed, rec_stride ) ) { ref_tile_fini( &t ); return -1; }
  memset( metrics, 0, 5UL*sizeof(ulong) );
  for( ulong i=0UL; i<n; i++ ) {
    /* during_frag: the frag lands in the out dcache chunk as an fd_txn_m_t record */
    fd_txn_m_t * txnm = (fd_txn_m_t *)t.buf;
    memset( txnm, 0, sizeof(fd_txn_m_t) );
    txnm->payload_sz = sz[i];
    txnm->block_engine.bundle_id = bid[i];
    memcpy( fd_txn_m_payload( txnm ), arena + off[i], sz[i] );
    rec_sz[i] = 0UL; tag[i] = 0UL;
    res[i] = ref_after_frag( &t, rec_sz + i, tag + i );
    if( res[i]==R_PUBLISH ) { memcpy( rec + i*rec_stride, t.buf, rec_sz[i] ); metrics[4]++; }
  }
  metrics[0] = t.ctx->metrics.parse_fail_cnt; metrics[1] = t.ctx->metrics.verify_fail_cnt;
  metrics[2] = t.ctx->metrics.dedup_fail_cnt; metrics[3] = t.ctx->metrics.bundle_peer_fail_cnt;
  ref_tile_fini( &t );
  return 0;
}
