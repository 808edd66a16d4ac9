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
   after_frag's bundle bookkeeping, restated statement for statement from
   src/disco/verify/fd_verify_tile.c:103-157 (after_frag is a static
   function of the tile's translation unit, which needs the stem and topo
   runtime).  libfdref_tile.so is the expectation of
   tests/test_gpu_vtile.py: every frag's outcome, the four metrics and the
   published fd_txn_m_t records. */

#include <limits.h>
#include <stdlib.h>
#include <string.h>
#include "disco/verify/fd_verify_tile.h"
#include "disco/fd_txn_m_t.h"
#include "ballet/txn/fd_txn.h"
#include "ballet/ed25519/fd_ed25519.h"

/* outcomes, as include/fd_verify_gpu.h's FDGPU_VTILE_* */
#define R_PUBLISH 0
#define R_PARSE   1
#define R_VERIFY  2
#define R_DEDUP   3
#define R_PEER    4

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
  fd_verify_ctx_t * ctx = (fd_verify_ctx_t *)calloc( 1, sizeof(fd_verify_ctx_t) );
  fd_sha512_t * sha = (fd_sha512_t *)aligned_alloc( FD_SHA512_ALIGN, FD_TXN_ACTUAL_SIG_MAX * sizeof(fd_sha512_t) );
  ulong map_cnt = fd_tcache_map_cnt_default( depth );
  ulong * ring = (ulong *)malloc( depth * sizeof(ulong) );
  ulong * map  = (ulong *)malloc( map_cnt * sizeof(ulong) );
  uchar * buf  = (uchar *)aligned_alloc( 64, rec_stride );
  if( !ctx || !sha || !ring || !map || !buf || !map_cnt ) { free( ctx ); free( sha ); free( ring ); free( map ); free( buf ); return -1; }
  for( ulong i=0UL; i<FD_TXN_ACTUAL_SIG_MAX; i++ ) ctx->sha[i] = fd_sha512_init( sha + i );
  ulong oldest = fd_tcache_reset( ring, depth, map, map_cnt );
  ctx->tcache_depth = depth; ctx->tcache_map_cnt = map_cnt;
  ctx->tcache_sync = &oldest; ctx->tcache_ring = ring; ctx->tcache_map = map;
  ctx->hashmap_seed = seed;
  memset( metrics, 0, 5UL*sizeof(ulong) );
  for( ulong i=0UL; i<n; i++ ) {
    /* during_frag: the frag lands in the out dcache chunk as an fd_txn_m_t record */
    fd_txn_m_t * txnm = (fd_txn_m_t *)buf;
    memset( txnm, 0, sizeof(fd_txn_m_t) );
    txnm->payload_sz = sz[i];
    txnm->block_engine.bundle_id = bid[i];
    memcpy( fd_txn_m_payload( txnm ), arena + off[i], sz[i] );
    res[i] = -1; rec_sz[i] = 0UL; tag[i] = 0UL;

    /* after_frag, fd_verify_tile.c:114-156 */
    fd_txn_t * txnt = fd_txn_m_txn_t( txnm );
    txnm->txn_t_sz = (ushort)fd_txn_parse( fd_txn_m_payload( txnm ), txnm->payload_sz, txnt, NULL );
    int is_bundle = !!txnm->block_engine.bundle_id;
    if( is_bundle & (txnm->block_engine.bundle_id!=ctx->bundle_id) ) {
      ctx->bundle_failed = 0;
      ctx->bundle_id     = txnm->block_engine.bundle_id;
    }
    if( is_bundle & (!!ctx->bundle_failed) ) { ctx->metrics.bundle_peer_fail_cnt++; res[i] = R_PEER; continue; }
    if( !txnm->txn_t_sz ) {
      if( is_bundle ) ctx->bundle_failed = 1;
      ctx->metrics.parse_fail_cnt++; res[i] = R_PARSE; continue;
    }
    ulong txn_sig = 0UL;
    int r = fd_txn_verify( ctx, fd_txn_m_payload( txnm ), txnm->payload_sz, txnt, !is_bundle, &txn_sig );
    if( r!=FD_TXN_VERIFY_SUCCESS ) {
      if( is_bundle ) ctx->bundle_failed = 1;
      if( r==FD_TXN_VERIFY_DEDUP ) { ctx->metrics.dedup_fail_cnt++; res[i] = R_DEDUP; }
      else                         { ctx->metrics.verify_fail_cnt++; res[i] = R_VERIFY; }
      continue;
    }
    ulong realized_sz = fd_txn_m_realized_footprint( txnm, 1, 0 );
    res[i] = R_PUBLISH; rec_sz[i] = realized_sz; tag[i] = is_bundle ? 0UL : txn_sig;
    memcpy( rec + i*rec_stride, buf, realized_sz );
    metrics[4]++;
  }
  metrics[0] = ctx->metrics.parse_fail_cnt; metrics[1] = ctx->metrics.verify_fail_cnt;
  metrics[2] = ctx->metrics.dedup_fail_cnt; metrics[3] = ctx->metrics.bundle_peer_fail_cnt;
  free( ctx ); free( sha ); free( ring ); free( map ); free( buf );
  return 0;
}
