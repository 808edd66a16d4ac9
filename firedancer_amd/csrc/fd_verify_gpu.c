/* fd_verify_gpu.c -- the verify tile's frag callbacks over the GPU engine,
   a minimal tango (mcache / dcache / tcache) and the streaming benchmark.
   Host C; see include/fd_verify_gpu.h for the contract and the reference
   lines each part replaces. */

#define _GNU_SOURCE
#include "../../include/fd_verify_gpu.h"
#include "../../include/fd_ed25519_gpu.h"

#include <pthread.h>
#include <stdio.h>
#include <stdatomic.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#if defined(__x86_64__)
#include <immintrin.h>
#endif

typedef unsigned long ulong;
typedef unsigned char uchar;

static ulong now_ns( void ) {
  struct timespec ts; clock_gettime( CLOCK_MONOTONIC, &ts );
  return (ulong)ts.tv_sec * 1000000000UL + (ulong)ts.tv_nsec;
}

static ulong pow2_up( ulong x ) { ulong p = 1UL; while( p < x ) p <<= 1; return p; }

/* ---- dedup tag: XXH64 of the first signature -----------------------
   fd_txn_verify tags a transaction with fd_hash( seed, sig0, 64 )
   (src/disco/verify/fd_verify_tile.h:79); fd_hash is XXH64 (r39), so
   this is the published XXH64 algorithm specialised to 64-byte input. */

#define P1 0x9E3779B185EBCA87UL
#define P2 0xC2B2AE3D27D4EB4FUL
#define P3 0x165667B19E3779F9UL
#define P4 0x85EBCA77C2B2AE63UL
#define P5 0x27D4EB2F165667C5UL

static ulong rotl64( ulong x, int r ) { return (x << r) | (x >> (64 - r)); }
static ulong ld64( uchar const * p ) { ulong x; memcpy( &x, p, 8 ); return x; }
static ulong xxh_round( ulong acc, ulong in ) { acc += in * P2; acc = rotl64( acc, 31 ); return acc * P1; }

static ulong
xxh64_64( ulong seed, uchar const * p ) {
  ulong v[4] = { seed + P1 + P2, seed + P2, seed, seed - P1 };
  for( int blk=0; blk<2; blk++ )
    for( int i=0; i<4; i++ ) v[i] = xxh_round( v[i], ld64( p + 32*blk + 8*i ) );
  ulong h = rotl64( v[0], 1 ) + rotl64( v[1], 7 ) + rotl64( v[2], 12 ) + rotl64( v[3], 18 );
  for( int i=0; i<4; i++ ) { h ^= xxh_round( 0UL, v[i] ); h = h * P1 + P4; }
  h += 64UL;
  h ^= h >> 33; h *= P2; h ^= h >> 29; h *= P3; h ^= h >> 32;
  return h;
}

ulong fdgpu_dedup_tag( ulong seed, uchar const sig[ 64 ] ) { return xxh64_64( seed, sig ); }

/* ---- tcache ----------------------------------------------------------
   Semantics of FD_TCACHE_QUERY / FD_TCACHE_INSERT (src/tango/tcache/
   fd_tcache.h:281-404): a ring of the last depth unique tags plus an
   open-addressed (linear probe) map; inserting a new tag evicts the
   oldest.  Tag 0 is the null tag (a query for it always "finds" it). */

struct fdgpu_tcache {
  ulong depth, map_cnt, oldest;
  ulong * ring;
  ulong * map;
};

static ulong tc_slot( ulong tag, ulong map_cnt ) { return (tag * P1 >> 17) & (map_cnt - 1UL); }

fdgpu_tcache_t *
fdgpu_tcache_new( ulong depth ) {
  if( !depth ) return NULL;
  fdgpu_tcache_t * tc = (fdgpu_tcache_t *)calloc( 1, sizeof(fdgpu_tcache_t) );
  if( !tc ) return NULL;
  tc->depth = depth; tc->map_cnt = pow2_up( 2UL*depth + 2UL ); tc->oldest = 0UL;
  tc->ring = (ulong *)calloc( depth, sizeof(ulong) );
  tc->map  = (ulong *)calloc( tc->map_cnt, sizeof(ulong) );
  if( !tc->ring || !tc->map ) { free( tc->ring ); free( tc->map ); free( tc ); return NULL; }
  return tc;
}

void fdgpu_tcache_delete( fdgpu_tcache_t * tc ) { if( tc ) { free( tc->ring ); free( tc->map ); free( tc ); } }

static int tc_find( fdgpu_tcache_t const * tc, ulong tag, ulong * idx ) {
  ulong i = tc_slot( tag, tc->map_cnt );
  for( ;; ) {
    ulong m = tc->map[i];
    if( m==tag ) { *idx = i; return 1; }
    if( !m )     { *idx = i; return 0; }
    i = (i + 1UL) & (tc->map_cnt - 1UL);
  }
}

int fdgpu_tcache_query( fdgpu_tcache_t const * tc, ulong tag ) {
  if( !tag ) return 1;
  ulong i; return tc_find( tc, tag, &i );
}

/* delete map slot i keeping every probe chain intact (backward shift) */
static void tc_map_remove( fdgpu_tcache_t * tc, ulong i ) {
  ulong mask = tc->map_cnt - 1UL;
  ulong j = i;
  for( ;; ) {
    j = (j + 1UL) & mask;
    ulong t = tc->map[j];
    if( !t ) break;
    ulong home = tc_slot( t, tc->map_cnt );
    /* move t into the hole at i unless its home lies cyclically in (i, j] */
    int stay = ( i <= j ) ? ( home > i && home <= j ) : ( home > i || home <= j );
    if( !stay ) { tc->map[i] = t; i = j; }
  }
  tc->map[i] = 0UL;
}

int fdgpu_tcache_insert( fdgpu_tcache_t * tc, ulong tag ) {
  if( !tag ) return 1;
  ulong i;
  if( tc_find( tc, tag, &i ) ) return 1;
  tc->map[i] = tag;
  ulong old = tc->ring[ tc->oldest ];
  tc->ring[ tc->oldest ] = tag;
  tc->oldest = ( tc->oldest + 1UL == tc->depth ) ? 0UL : tc->oldest + 1UL;
  if( old && tc_find( tc, old, &i ) ) tc_map_remove( tc, i );
  return 0;
}

/* ---- mcache / dcache -------------------------------------------------
   An mcache is a ring of frag metadata indexed by seq & (depth-1); the
   producer writes the entry and then its seq (release); a consumer
   waiting for seq reads the entry between two acquire loads of its seq
   field and classifies: equal = ready, behind = not yet published,
   ahead = overrun (src/tango/mcache/fd_mcache.h:288-325 semantics). */

typedef struct {
  _Atomic ulong     seq;
  fdgpu_frag_meta_t m;
} mc_line_t;

struct fdgpu_mcache {
  ulong       depth;
  mc_line_t * line;
};

fdgpu_mcache_t *
fdgpu_mcache_new( ulong depth, ulong seq0 ) {
  if( !depth || (depth & (depth - 1UL)) ) return NULL;
  fdgpu_mcache_t * mc = (fdgpu_mcache_t *)calloc( 1, sizeof(fdgpu_mcache_t) );
  if( !mc ) return NULL;
  mc->depth = depth;
  mc->line = (mc_line_t *)aligned_alloc( 64, depth * sizeof(mc_line_t) + 64 );
  if( !mc->line ) { free( mc ); return NULL; }
  memset( mc->line, 0, depth * sizeof(mc_line_t) );
  /* every line starts "one lap behind" so seq0.. read as not yet published */
  for( ulong i=0; i<depth; i++ ) atomic_store_explicit( &mc->line[i].seq, seq0 + i - depth, memory_order_relaxed );
  return mc;
}

void fdgpu_mcache_delete( fdgpu_mcache_t * mc ) { if( mc ) { free( mc->line ); free( mc ); } }

void
fdgpu_mcache_publish( fdgpu_mcache_t * mc, ulong seq, ulong sig, unsigned chunk, unsigned sz, ulong tsorig, ulong tspub ) {
  mc_line_t * l = &mc->line[ seq & (mc->depth - 1UL) ];
  atomic_store_explicit( &l->seq, seq - 1UL, memory_order_relaxed );   /* mark in-progress */
  atomic_thread_fence( memory_order_release );
  l->m.seq = seq; l->m.sig = sig; l->m.chunk = chunk; l->m.sz = sz; l->m.tsorig = tsorig; l->m.tspub = tspub;
  atomic_store_explicit( &l->seq, seq, memory_order_release );
}

int
fdgpu_mcache_poll( fdgpu_mcache_t const * mc, ulong seq, fdgpu_frag_meta_t * out ) {
  mc_line_t const * l = &mc->line[ seq & (mc->depth - 1UL) ];
  ulong s0 = atomic_load_explicit( (_Atomic ulong *)&l->seq, memory_order_acquire );
  if( (long)(s0 - seq) < 0 ) return 1;
  if( s0 != seq ) return -1;
  fdgpu_frag_meta_t m = l->m;
  atomic_thread_fence( memory_order_acquire );
  ulong s1 = atomic_load_explicit( (_Atomic ulong *)&l->seq, memory_order_relaxed );
  if( s1 != seq ) return -1;
  *out = m;
  return 0;
}

/* fd_dcache_compact_next (src/tango/dcache/fd_dcache.h:263-269): advance
   by whole 128-byte chunk pairs, wrap to chunk0 past wmark */
ulong
fdgpu_dcache_compact_next( ulong chunk, ulong sz, ulong chunk0, ulong wmark ) {
  chunk += ( ( sz + 2UL*FDGPU_CHUNK_SZ - 1UL ) >> 7 ) << 1;
  return chunk > wmark ? chunk0 : chunk;
}

/* ---- the verify tile ------------------------------------------------ */

/* during_frag's copy into the out dcache.  The GPU reads the payload by
   DMA and after_frag comes back to the record only milliseconds later, so
   the bulk goes out with non-temporal stores (no read-for-ownership of
   destination lines that would be evicted before their next use).
   vt_fence() makes them visible before anything that can launch a batch:
   at the top of during_frag (a launch inside submit_raw_ref only uploads
   earlier frags), housekeep, flush and blocking drains. */
static void
vt_copy( uchar * dst, uchar const * src, ulong sz ) {
#if defined(__x86_64__)
  ulong n16 = sz & ~15UL;                         /* dst is chunk (64-B) aligned */
  for( ulong i=0UL; i<n16; i+=16UL )
    _mm_stream_si128( (__m128i *)( dst + i ), _mm_loadu_si128( (__m128i const *)( src + i ) ) );
  if( sz > n16 ) memcpy( dst + n16, src + n16, sz - n16 );
#else
  memcpy( dst, src, sz );
#endif
}

static inline void
vt_fence( void ) {
#if defined(__x86_64__)
  _mm_sfence();
#else
  atomic_thread_fence( memory_order_seq_cst );
#endif
}

#define VT_RESERVE_MAX ( FDGPU_TXNM_HDR_SZ + 1232UL + 2UL + 852UL )   /* header + MTU payload + fd_txn_t */

typedef struct {
  ulong seq, tsorig, chunk;
  int   k;                               /* engine context the frag's batch went to */
} vt_pend_t;

/* Engine contexts per tile (env FDGPU_VTILE_CTX, 1..VT_NCTX_MAX, default 2).
   A context runs its batches in order on one HIP stream, so with one
   context a frag that arrives while a batch runs waits for all of it.
   With several, the tile fills them in turn and launches staggered by
   the batch duration / nctx, so batches overlap on the GPU and a frag
   waits for at most that stagger before its batch starts.  Completions
   are merged back into frag order in after_frags. */
#define VT_NCTX_MAX 3

struct fdgpu_vtile {
  /* (fields below; ctx first so the watchdog can report pipeline state) */
  fdgpu_ed25519_ctx_t * ctx[ VT_NCTX_MAX ];
  int                   nctx, fill;      /* contexts, the one taking frags */
  ulong                 launch_ns[ VT_NCTX_MAX ];
  int                   busy[ VT_NCTX_MAX ];
  double                batch_ns;        /* EWMA of launch -> drained */
  fdgpu_tcache_t *      tcache;
  ulong                 seed;
  uchar *               dcache;
  ulong                 chunk0, wmark, out_chunk;
  vt_pend_t *           pend;            /* FIFO of frags between during_frag and after_frags */
  ulong                 pend_cap, pend_head, pend_tail;   /* monotonic counters */
  int                   bundle_failed;
  ulong                 bundle_id;
  ulong                 metrics[5];
  /* zero-copy intake (fdgpu_vtile_set_in_link): frags stay in the in
     dcache, the GPU gathers them; in_mc (optional) for the overrun check */
  int                   zc;
  fdgpu_mcache_t const * in_mc;
  ulong                 overruns;
  /* poll scratch */
  ulong                 batch;
  ulong *               p_tags;
  signed char *         p_codes;
  uchar *               p_img;
  unsigned short *      p_fp;
};

fdgpu_vtile_t *
fdgpu_vtile_new( int device, ulong batch_txn, ulong tcache_depth, ulong seed, ulong out_dcache_bytes, int semantics ) {
  if( !batch_txn || !tcache_depth || out_dcache_bytes < 8UL*VT_RESERVE_MAX ) return NULL;
  fdgpu_vtile_t * vt = (fdgpu_vtile_t *)calloc( 1, sizeof(fdgpu_vtile_t) );
  if( !vt ) return NULL;
  /* staging arena of a batch = its range of the out dcache (in-place submits): up to
     batch_txn records of at most VT_RESERVE_MAX bytes (rounded to chunk pairs) */
  char const * ne = getenv( "FDGPU_VTILE_CTX" );
  vt->nctx = ne ? atoi( ne ) : 2;
  if( vt->nctx < 1 ) vt->nctx = 1;
  if( vt->nctx > VT_NCTX_MAX ) vt->nctx = VT_NCTX_MAX;
  vt->batch_ns = 500e3;
  int ctx_ok = 1;
  for( int k=0; k<vt->nctx; k++ ) {
    vt->ctx[k] = fdgpu_ed25519_ctx_new( device, batch_txn, 16UL*batch_txn, batch_txn*2304UL + 1024UL, semantics );
    /* adaptive batching launches a partial batch when the GPU has room (low
       load: the latency path) and a full one when frags back up (high load:
       the throughput path, whose per-signature work is 0.5x the 4-lane DSM's) */
    if( vt->ctx[k] ) {
      ulong sm = fdgpu_ed25519_set_small_batch_max( vt->ctx[k], 0UL );
      fdgpu_ed25519_set_small_batch_max( vt->ctx[k], sm < batch_txn/2UL ? sm : batch_txn/2UL );
    } else ctx_ok = 0;
  }
  vt->tcache = fdgpu_tcache_new( tcache_depth );
  ulong nchunk = ( out_dcache_bytes / FDGPU_CHUNK_SZ ) & ~1UL;
  vt->dcache = (uchar *)fdgpu_host_alloc( nchunk * FDGPU_CHUNK_SZ );   /* pinned: batches upload from it in place */
  ulong rchunk = ( ( VT_RESERVE_MAX + 127UL ) >> 7 ) << 1;
  vt->chunk0 = 0UL; vt->wmark = nchunk - rchunk; vt->out_chunk = 0UL;
  /* frags in flight: the ring must hold them all plus one wrap's waste */
  vt->pend_cap = nchunk / rchunk - 2UL;
  vt->pend = (vt_pend_t *)calloc( vt->pend_cap, sizeof(vt_pend_t) );
  vt->seed = seed;
  vt->batch = batch_txn;
  vt->p_tags = (ulong *)malloc( batch_txn * sizeof(ulong) );
  vt->p_codes = (signed char *)malloc( batch_txn );
  vt->p_img = (uchar *)malloc( batch_txn * FDGPU_TXN_IMG_STRIDE );
  vt->p_fp = (unsigned short *)malloc( batch_txn * sizeof(unsigned short) );
  if( !ctx_ok || !vt->tcache || !vt->dcache || !vt->pend || !vt->p_tags || !vt->p_codes || !vt->p_img || !vt->p_fp ) {
    fdgpu_vtile_delete( vt );
    return NULL;
  }
  return vt;
}

void
fdgpu_vtile_delete( fdgpu_vtile_t * vt ) {
  if( !vt ) return;
  for( int k=0; k<VT_NCTX_MAX; k++ ) if( vt->ctx[k] ) fdgpu_ed25519_ctx_delete( vt->ctx[k] );
  fdgpu_tcache_delete( vt->tcache );
  fdgpu_host_free( vt->dcache ); free( vt->pend ); free( vt->p_tags ); free( vt->p_codes ); free( vt->p_img ); free( vt->p_fp );
  free( vt );
}

uchar * fdgpu_vtile_out_dcache( fdgpu_vtile_t * vt ) { return vt->dcache; }
ulong   fdgpu_vtile_pending( fdgpu_vtile_t const * vt ) { return vt->pend_tail - vt->pend_head; }
void    fdgpu_vtile_metrics( fdgpu_vtile_t const * vt, ulong out[ 5 ] ) { memcpy( out, vt->metrics, sizeof(vt->metrics) ); }
int
fdgpu_vtile_flush( fdgpu_vtile_t * vt ) {
  vt_fence();
  int rc = 0;
  for( int i=0; i<vt->nctx; i++ ) {            /* oldest first: the fill context's batch is the newest */
    int k = ( vt->fill + 1 + i ) % vt->nctx;
    ulong filling, inflight;
    fdgpu_ed25519_pipeline_state( vt->ctx[k], &filling, &inflight );
    if( !filling ) continue;
    if( fdgpu_ed25519_flush( vt->ctx[k] ) ) rc = -1;
    else { vt->launch_ns[k] = now_ns(); vt->busy[k] = 1; }
  }
  return rc;
}

void
fdgpu_vtile_pipeline_state( fdgpu_vtile_t const * vt, ulong * filling, ulong * inflight ) {
  *filling = 0UL; *inflight = 0UL;
  for( int k=0; k<vt->nctx; k++ ) {
    ulong f, i;
    fdgpu_ed25519_pipeline_state( vt->ctx[k], &f, &i );
    *filling += f; *inflight += i;
  }
}
ulong   fdgpu_vtile_overruns( fdgpu_vtile_t const * vt ) { return vt->overruns; }

int
fdgpu_vtile_set_in_link( fdgpu_vtile_t * vt, fdgpu_mcache_t const * in_mc ) {
  if( vt->pend_tail != vt->pend_head ) return -1;       /* switch only while idle */
  vt->zc = 1; vt->in_mc = in_mc;
  return 0;
}

ulong
fdgpu_vtile_oldest_pending_seq( fdgpu_vtile_t const * vt ) {
  return vt->pend_head < vt->pend_tail ? vt->pend[ vt->pend_head % vt->pend_cap ].seq : ~0UL;
}

int
fdgpu_vtile_housekeep( fdgpu_vtile_t * vt, ulong max_inflight ) {
  ulong filling, inflight, now = now_ns();
  /* batch duration: a context's batches have drained (inflight counts
     launched slots not yet fully polled) */
  for( int k=0; k<vt->nctx; k++ ) {
    if( !vt->busy[k] ) continue;
    ulong f, i;
    fdgpu_ed25519_pipeline_state( vt->ctx[k], &f, &i );
    if( !i ) { vt->busy[k] = 0; vt->batch_ns = 0.875*vt->batch_ns + 0.125*(double)( now - vt->launch_ns[k] ); }
  }
  int f = vt->fill;
  fdgpu_ed25519_pipeline_state( vt->ctx[f], &filling, &inflight );
  /* keep at least one staging slot free to accumulate in: with every slot
     in flight, each freed slot would be relaunched after a handful of
     frags and the pipeline would degenerate into tiny batches */
  if( max_inflight > 3UL ) max_inflight = 3UL;
  if( !filling || inflight >= max_inflight ) return 0;
  if( vt->nctx > 1 && filling < vt->batch ) {
    /* stagger: launch once every other context's newest batch has run
       batch_ns / nctx (or that context is idle) */
    ulong stagger = (ulong)( vt->batch_ns / (double)vt->nctx );
    for( int k=0; k<vt->nctx; k++ )
      if( k != f && vt->busy[k] && now - vt->launch_ns[k] < stagger ) return 0;
  }
  vt_fence();
  if( fdgpu_ed25519_flush( vt->ctx[f] ) ) return 0;
  vt->launch_ns[f] = now; vt->busy[f] = 1;
  vt->fill = ( f + 1 ) % vt->nctx;
  return 1;
}

int
fdgpu_vtile_during_frag( fdgpu_vtile_t * vt, void const * frag, ulong sz, ulong seq, ulong tsorig ) {
  fdgpu_txnm_t const * in = (fdgpu_txnm_t const *)frag;
  /* fd_verify_tile.c:78-85: the frag must hold its header + payload and
     the payload must fit the MTU (the reference FD_LOG_ERRs) */
  if( sz < FDGPU_TXNM_HDR_SZ || in->payload_sz > 1232U || FDGPU_TXNM_HDR_SZ + in->payload_sz > sz ) return -4;
  vt_fence();
  if( vt->pend_tail - vt->pend_head >= vt->pend_cap ) { fdgpu_vtile_flush( vt ); return -2; }
  uchar * dst = vt->dcache + vt->out_chunk * FDGPU_CHUNK_SZ;
  int rc;
  if( vt->zc ) {   /* the GPU copies the frag into dst itself (no host copy) */
    rc = fdgpu_ed25519_submit_raw_gather( vt->ctx[ vt->fill ], (uchar const *)frag, vt->dcache, dst,
                                          (unsigned short)( FDGPU_TXNM_HDR_SZ + in->payload_sz ),
                                          (unsigned short)FDGPU_TXNM_HDR_SZ, in->payload_sz, vt->pend_tail );
  } else {
    vt_copy( dst, (uchar const *)frag, FDGPU_TXNM_HDR_SZ + in->payload_sz );
    rc = fdgpu_ed25519_submit_raw_ref( vt->ctx[ vt->fill ], vt->dcache, dst + FDGPU_TXNM_HDR_SZ, in->payload_sz, vt->pend_tail );
  }
  if( rc ) return rc;
  vt_pend_t * p = &vt->pend[ vt->pend_tail % vt->pend_cap ];
  p->seq = seq; p->tsorig = tsorig; p->chunk = vt->out_chunk; p->k = vt->fill;
  vt->pend_tail++;
  ulong reserve = ( ( FDGPU_TXNM_HDR_SZ + in->payload_sz + 1UL ) & ~1UL ) + 852UL;
  vt->out_chunk = fdgpu_dcache_compact_next( vt->out_chunk, reserve, vt->chunk0, vt->wmark );
  return 0;
}

/* after_frag (fd_verify_tile.c:103-157) for one completed frag */
static int
vt_after( fdgpu_vtile_t * vt, vt_pend_t const * p, int code, uchar const * img, unsigned fp, fdgpu_vtile_done_t * d ) {
  fdgpu_txnm_t * txnm = (fdgpu_txnm_t *)( vt->dcache + p->chunk * FDGPU_CHUNK_SZ );
  uchar * payload = (uchar *)txnm + FDGPU_TXNM_HDR_SZ;
  d->seq = p->seq; d->tsorig = p->tsorig; d->chunk = p->chunk; d->sz = 0UL; d->tag = 0UL;
  if( vt->zc && vt->in_mc ) {
    /* zero-copy: the GPU read the frag at batch launch, after during_frag.
       If the producer has since reused the frag's mcache line, its dcache
       bytes may have been overwritten before that read: drop it, as the
       stem loop drops a frag overrun during its copy. */
    fdgpu_frag_meta_t m;
    if( fdgpu_mcache_poll( vt->in_mc, p->seq, &m ) != 0 ) { vt->overruns++; return FDGPU_VTILE_OVERRUN; }
  }
  txnm->txn_t_sz = (unsigned short)fp;
  int is_bundle = txnm->bundle_id != 0UL;
  if( is_bundle && txnm->bundle_id != vt->bundle_id ) { vt->bundle_failed = 0; vt->bundle_id = txnm->bundle_id; }
  if( is_bundle && vt->bundle_failed ) { vt->metrics[3]++; return FDGPU_VTILE_BUNDLE_PEER_FAIL; }
  if( code == FDGPU_ERR_PARSE ) {
    if( is_bundle ) vt->bundle_failed = 1;
    vt->metrics[0]++;
    return FDGPU_VTILE_PARSE_FAIL;
  }
  /* zero-copy: the GPU already wrote the fd_txn_t image behind the payload */
  ulong t_off = ( FDGPU_TXNM_HDR_SZ + txnm->payload_sz + 1UL ) & ~1UL;
  if( vt->zc ) img = (uchar const *)txnm + t_off;
  /* fd_txn_verify (fd_verify_tile.h:59-108): dedup query, verify, insert */
  unsigned sig_off = (unsigned)img[2] | ((unsigned)img[3] << 8);
  ulong tag = xxh64_64( vt->seed, payload + sig_off );
  int res = 0;   /* 0 success, 1 verify failed, 2 dedup */
  if( !is_bundle && fdgpu_tcache_query( vt->tcache, tag ) ) res = 2;
  else if( code != 0 ) res = 1;
  else if( !is_bundle && fdgpu_tcache_insert( vt->tcache, tag ) ) res = 2;
  if( res ) {
    if( is_bundle ) vt->bundle_failed = 1;
    if( res==2 ) { vt->metrics[2]++; return FDGPU_VTILE_DEDUP_FAIL; }
    vt->metrics[1]++;
    return FDGPU_VTILE_VERIFY_FAIL;
  }
  /* publish: fd_txn_t behind the payload at a 2-byte boundary */
  if( !vt->zc ) memcpy( (uchar *)txnm + t_off, img, fp );
  d->sz = t_off + fp;                                  /* fd_txn_m_realized_footprint( txnm, 1, 0 ) */
  d->tag = is_bundle ? 0UL : tag;
  vt->metrics[4]++;
  return FDGPU_VTILE_PUBLISH;
}

ulong
fdgpu_vtile_after_frags( fdgpu_vtile_t * vt, fdgpu_vtile_done_t * out, ulong max, int blocking ) {
  ulong n = 0UL;
  if( blocking ) fdgpu_vtile_flush( vt );      /* a blocking drain must not wait on an unlaunched batch */
  while( n < max && vt->pend_head < vt->pend_tail ) {
    /* the next completions in frag order: the run of pending frags from
       the head that went to the same context (each context completes in
       its own submission order) */
    int c = vt->pend[ vt->pend_head % vt->pend_cap ].k;
    ulong want = 1UL, lim = max - n;
    if( lim > vt->batch ) lim = vt->batch;
    while( want < lim && vt->pend_head + want < vt->pend_tail &&
           vt->pend[ ( vt->pend_head + want ) % vt->pend_cap ].k == c ) want++;
    ulong k = fdgpu_ed25519_poll_raw( vt->ctx[c], vt->p_tags, vt->p_codes, vt->zc ? NULL : vt->p_img, vt->p_fp, want, blocking );
    if( !k ) break;
    for( ulong i=0; i<k; i++ ) {
      /* the records were written by the GPU / by non-temporal stores, so they are not in
         this core's caches: prefetch a few frags ahead -- header + first signature lines at
         distance 8, the fd_txn_t line (its offset needs the header) at distance 4 */
      if( vt->pend_head + 8UL < vt->pend_tail ) {
        uchar const * r = vt->dcache + vt->pend[ ( vt->pend_head + 8UL ) % vt->pend_cap ].chunk * FDGPU_CHUNK_SZ;
        __builtin_prefetch( r ); __builtin_prefetch( r + 64 ); __builtin_prefetch( r + 128 );
      }
      if( vt->pend_head + 4UL < vt->pend_tail ) {
        uchar const * r = vt->dcache + vt->pend[ ( vt->pend_head + 4UL ) % vt->pend_cap ].chunk * FDGPU_CHUNK_SZ;
        __builtin_prefetch( r + ( ( FDGPU_TXNM_HDR_SZ + ((fdgpu_txnm_t const *)r)->payload_sz + 1UL ) & ~1UL ) );
      }
      vt_pend_t const * p = &vt->pend[ vt->pend_head % vt->pend_cap ];
      /* tags are the pending counter: completions come back in order */
      out[n].result = vt_after( vt, p, (int)vt->p_codes[i], vt->p_img + i*FDGPU_TXN_IMG_STRIDE, vt->p_fp[i], &out[n] );
      vt->pend_head++; n++;
    }
    blocking = 0;
  }
  return n;
}

/* ---- streaming benchmark -------------------------------------------- */

typedef struct {
  /* shared */
  fdgpu_mcache_t *       mc;
  uchar *                in_dcache;
  ulong                  in_chunk0, in_wmark;
  ulong                  n_frags;
  int                    tiles;
  struct { _Atomic ulong v; uchar pad[56]; } * fseq;   /* per tile, own cache line: next seq it has yet to consume */
  _Atomic int            go, fail, ready;
  ulong *                lh;          /* merged latency histogram (lh_idx buckets) */
  ulong                  lmax;        /* max latency, ns */
  unsigned char const *  payload; unsigned int const * off; unsigned short const * sz; ulong n_payload;
  ulong *                frag_chunk;  /* in dcache chunk of payload p's prefilled frag record */
  double                 rate_fps;
  ulong                  depth;
  ulong                  t_start, t_end;
  _Atomic ulong          t_last;
  _Atomic ulong          sigs, published, overruns;
  _Atomic ulong          ns[4];        /* summed over tiles: during_frag, after_frags, housekeep, loop total */
  ulong                  metrics[5];
  pthread_mutex_t        mu;
  int                    device; ulong batch_txn, max_inflight;
  int                    zc;          /* zero-copy intake: tiles leave frags in the in dcache */
} sb_t;

/* The producer stands in for the QUIC tiles: every distinct payload is
   written once, before the run, into the in dcache as an fd_txn_m_t frag
   record (as the NIC / QUIC reassembly would have left it), and the
   timed loop only publishes metadata -- frag seq points at payload
   seq % n_payload.  The link is reliable (credit based): the producer
   runs at most depth/2 frags ahead of the slowest tile, re-reading the
   tiles' fseqs only when its cached credits run out. */
static void * sb_producer( void * _s ) {
  sb_t * s = (sb_t *)_s;
  while( !atomic_load( &s->go ) ) ;
  ulong t0 = now_ns();
  s->t_start = t0;
  ulong cr_until = 0UL;                     /* may publish seq < cr_until */
  for( ulong seq=0; seq<s->n_frags; seq++ ) {
    ulong t_wait = 0UL;
    while( seq >= cr_until ) {
      if( atomic_load_explicit( &s->fail, memory_order_relaxed ) ) return NULL;
      if( !t_wait ) t_wait = now_ns();
      else if( now_ns() - t_wait > 30000000000UL ) {            /* watchdog: 30 s without credits */
        fprintf( stderr, "fdgpu_stream_bench: producer starved of credits at seq %lu\n", seq );
        atomic_store( &s->fail, 4 ); return NULL;
      }
      ulong lo = ~0UL;
      for( int t=0; t<s->tiles; t++ ) { ulong f = atomic_load_explicit( &s->fseq[t].v, memory_order_acquire ); if( f < lo ) lo = f; }
      cr_until = lo + s->depth/2;
    }
    if( s->rate_fps > 0. ) {
      ulong due = t0 + (ulong)( (double)seq * 1e9 / s->rate_fps );
      while( now_ns() < due ) ;
    }
    ulong p = seq % s->n_payload;
    ulong ts = now_ns();
    fdgpu_mcache_publish( s->mc, seq, 0UL, (unsigned)s->frag_chunk[p], (unsigned)( FDGPU_TXNM_HDR_SZ + s->sz[p] ), ts, ts );
  }
  return NULL;
}

typedef struct { sb_t * s; int idx; } sb_tile_arg_t;

/* credit a tile returns to the producer: every seq below it may be
   overwritten.  With zero-copy intake a frag's bytes must survive until
   the GPU has read them, so the credit stops at the oldest frag still
   pending in the tile. */
static void sb_credit( sb_t * s, int idx, fdgpu_vtile_t const * vt, ulong seq ) {
  ulong c = seq;
  if( s->zc ) { ulong o = fdgpu_vtile_oldest_pending_seq( vt ); if( o < c ) c = o; }
  atomic_store_explicit( &s->fseq[idx].v, c, memory_order_release );
}

/* Latency histogram (per tile, merged at the end): log-linear buckets,
   64 per octave (< 1.6 % wide), exact below 64 ns. */
#define LH_SUB 64UL
#define LH_N   ( LH_SUB + 40UL*LH_SUB )
static ulong lh_idx( ulong ns ) {
  if( ns < LH_SUB ) return ns;
  ulong b = 63UL - (ulong)__builtin_clzl( ns );                  /* >= 6 */
  ulong i = LH_SUB + ( b - 6UL ) * LH_SUB + ( ( ns >> ( b - 6UL ) ) & ( LH_SUB - 1UL ) );
  return i < LH_N ? i : LH_N - 1UL;
}
static double lh_val( ulong i ) {                                   /* bucket midpoint, ns */
  if( i < LH_SUB ) return (double)i;
  ulong b = ( i - LH_SUB ) / LH_SUB + 6UL, sub = ( i - LH_SUB ) % LH_SUB;
  return ( (double)( LH_SUB + sub ) + 0.5 ) * (double)( 1UL << ( b - 6UL ) );
}
static double lh_quantile( ulong const * h, ulong tot, double q ) {
  ulong want = (ulong)( q * (double)tot ), cum = 0UL;
  if( want >= tot ) want = tot - 1UL;
  for( ulong i=0UL; i<LH_N; i++ ) { cum += h[i]; if( cum > want ) return lh_val( i ); }
  return lh_val( LH_N - 1UL );
}

static void sb_account( sb_t * s, fdgpu_vtile_t * vt, fdgpu_vtile_done_t const * d, ulong n, ulong * sigs,
                        ulong * lh, ulong * lmax ) {
  ulong t = now_ns();
  for( ulong i=0; i<n; i++ ) {
    ulong lat = t - d[i].tsorig;
    lh[ lh_idx( lat ) ]++;
    if( lat > *lmax ) *lmax = lat;
    if( d[i].result == FDGPU_VTILE_PUBLISH || d[i].result == FDGPU_VTILE_VERIFY_FAIL || d[i].result == FDGPU_VTILE_DEDUP_FAIL ) {
      uchar const * pl = fdgpu_vtile_out_dcache( vt ) + d[i].chunk * FDGPU_CHUNK_SZ + FDGPU_TXNM_HDR_SZ;
      *sigs += pl[0];
    }
  }
  if( n ) {
    ulong prev = atomic_load( &s->t_last );
    while( t > prev && !atomic_compare_exchange_weak( &s->t_last, &prev, t ) ) ;
  }
}

static void * sb_tile( void * _a ) {
  sb_tile_arg_t * a = (sb_tile_arg_t *)_a;
  sb_t * s = a->s;
  int idx = a->idx;
  fdgpu_vtile_t * vt = fdgpu_vtile_new( s->device, s->batch_txn, 1UL<<16, 0x5eedUL + (ulong)idx,
                                        ( 6UL*s->batch_txn + 64UL ) * 2304UL, FDGPU_SEMANTICS_AVX512 );
  if( !vt ) { atomic_store( &s->fail, 1 ); return NULL; }
  if( s->zc && fdgpu_vtile_set_in_link( vt, s->mc ) ) { atomic_store( &s->fail, 1 ); fdgpu_vtile_delete( vt ); return NULL; }
  atomic_fetch_add( &s->ready, 1 );              /* the producer starts once every tile has its GPU context */
  ulong dcap = 4096UL;
  fdgpu_vtile_done_t * done = (fdgpu_vtile_done_t *)malloc( dcap * sizeof(fdgpu_vtile_done_t) );
  ulong * lh = (ulong *)calloc( LH_N, sizeof(ulong) ), lmax = 0UL;
  ulong const T = (ulong)s->tiles;
  ulong sigs = 0UL, mine = 0UL, got = 0UL;
  for( ulong q=0; q<s->n_frags; q++ ) mine += ( q % T ) == (ulong)idx;
  ulong seq = 0UL;
  ulong last_seq = ~0UL, last_got = ~0UL, t_prog = now_ns();
  ulong t_hk = 0UL, ns_in = 0UL, ns_after = 0UL, ns_hk = 0UL, t_begin = now_ns();
  while( got < mine ) {
    if( atomic_load_explicit( &s->fail, memory_order_relaxed ) ) break;
    ulong t0 = now_ns();
    if( seq != last_seq || got != last_got ) { last_seq = seq; last_got = got; t_prog = t0; }
    else if( t0 - t_prog > 30000000000UL ) {                      /* watchdog: 30 s without progress */
      ulong filling = 0, inflight = 0;
      fdgpu_vtile_pipeline_state( vt, &filling, &inflight );
      fprintf( stderr, "fdgpu_stream_bench: tile %d stalled: seq %lu got %lu/%lu pending %lu filling %lu inflight %lu\n",
               idx, seq, got, mine, fdgpu_vtile_pending( vt ), filling, inflight );
      atomic_store( &s->fail, 5 ); break;
    }
    /* intake: up to 64 frags per pass.  Every seq's mcache line is read, as
       the stem loop does; before_frag keeps seq % tiles == idx. */
    int drain = 0;
    for( int k=0; k<64 && seq < s->n_frags; k++ ) {
      fdgpu_frag_meta_t m;
      int r = fdgpu_mcache_poll( s->mc, seq, &m );
      if( r > 0 ) break;
      if( r < 0 ) { atomic_fetch_add( &s->overruns, 1 ); atomic_store( &s->fail, 3 ); break; }
      if( ( seq % T ) == (ulong)idx ) {                             /* before_frag round robin */
        int rc = fdgpu_vtile_during_frag( vt, s->in_dcache + (ulong)m.chunk * FDGPU_CHUNK_SZ, m.sz, seq, m.tsorig );
        if( rc == -2 ) { drain = 1; break; }                        /* staging full: drain, retry this seq */
        if( rc ) { atomic_store( &s->fail, 2 ); break; }
        /* this tile's next frag is usually published already: start its cold lines */
        fdgpu_frag_meta_t nx;
        if( seq + T < s->n_frags && !fdgpu_mcache_poll( s->mc, seq + T, &nx ) ) {
          uchar const * pf = s->in_dcache + (ulong)nx.chunk * FDGPU_CHUNK_SZ;
          for( ulong o=0UL; o<nx.sz; o+=64UL ) __builtin_prefetch( pf + o );
        }
      }
      seq++;
      if( !(seq & 63UL) || seq==s->n_frags ) sb_credit( s, idx, vt, seq );   /* batched credit return */
    }
    ulong t1 = now_ns();
    ns_in += t1 - t0;
    if( atomic_load_explicit( &s->fail, memory_order_relaxed ) ) break;
    if( drain ) {
      ulong n = fdgpu_vtile_after_frags( vt, done, dcap, 1 );
      sb_account( s, vt, done, n, &sigs, lh, &lmax ); got += n;
      if( s->zc ) sb_credit( s, idx, vt, seq );
      ns_after += now_ns() - t1;
      continue;
    }
    /* housekeeping: launch / drain at most every 10 us while frags flow
       (the HIP runtime calls behind them take locks shared by all tiles) */
    if( t1 - t_hk >= 10000UL ) {
      t_hk = t1;
      fdgpu_vtile_housekeep( vt, s->max_inflight );                 /* adaptive batching */
      ulong t2 = now_ns();
      ulong n = fdgpu_vtile_after_frags( vt, done, dcap, 0 );
      sb_account( s, vt, done, n, &sigs, lh, &lmax ); got += n;
      if( s->zc && n ) sb_credit( s, idx, vt, seq );
      ns_hk += t2 - t1; ns_after += now_ns() - t2;
    }
  }
  ulong t_end = now_ns();
  atomic_fetch_add( &s->ns[0], ns_in );     atomic_fetch_add( &s->ns[1], ns_after );
  atomic_fetch_add( &s->ns[2], ns_hk );     atomic_fetch_add( &s->ns[3], t_end - t_begin );
  ulong m5[5]; fdgpu_vtile_metrics( vt, m5 );
  atomic_fetch_add( &s->overruns, fdgpu_vtile_overruns( vt ) );
  pthread_mutex_lock( &s->mu );
  for( int i=0; i<5; i++ ) s->metrics[i] += m5[i];
  for( ulong i=0UL; i<LH_N; i++ ) s->lh[i] += lh[i];
  if( lmax > s->lmax ) s->lmax = lmax;
  pthread_mutex_unlock( &s->mu );
  atomic_fetch_add( &s->sigs, sigs );
  free( done ); free( lh );
  fdgpu_vtile_delete( vt );
  return NULL;
}

int
fdgpu_stream_bench( int device, uchar const * payload, unsigned const * off, unsigned short const * sz, ulong n_payload,
                    ulong n_frags, int tiles, ulong batch_txn, ulong max_inflight, ulong mcache_depth, double rate_fps,
                    int zero_copy, fdgpu_stream_stats_t * st ) {
  if( tiles < 1 || tiles > 64 || !n_frags || !n_payload || !batch_txn || mcache_depth < 64 ) return -1;
  sb_t * s = (sb_t *)calloc( 1, sizeof(sb_t) );
  s->depth = pow2_up( mcache_depth );
  s->mc = fdgpu_mcache_new( s->depth, 0UL );
  /* in dcache: one prefilled fd_txn_m_t frag record per distinct payload */
  ulong in_bytes = 0UL;
  for( ulong p=0; p<n_payload; p++ ) in_bytes += ( ( FDGPU_TXNM_HDR_SZ + sz[p] + 127UL ) >> 7 ) << 7;
  s->in_dcache = (uchar *)aligned_alloc( 128, in_bytes + 128UL );
  s->frag_chunk = (ulong *)malloc( n_payload * sizeof(ulong) );
  if( !s->in_dcache || !s->frag_chunk ) { free( s->in_dcache ); free( s->frag_chunk ); fdgpu_mcache_delete( s->mc ); free( s ); return -2; }
  for( ulong p=0, c=0; p<n_payload; p++ ) {
    fdgpu_txnm_t * txnm = (fdgpu_txnm_t *)( s->in_dcache + c * FDGPU_CHUNK_SZ );
    memset( txnm, 0, FDGPU_TXNM_HDR_SZ );
    txnm->payload_sz = sz[p];
    memcpy( (uchar *)txnm + FDGPU_TXNM_HDR_SZ, payload + off[p], sz[p] );
    s->frag_chunk[p] = c;
    c = fdgpu_dcache_compact_next( c, FDGPU_TXNM_HDR_SZ + sz[p], 0UL, ~0UL );
  }
  s->n_frags = n_frags; s->tiles = tiles;
  s->fseq = calloc( (size_t)tiles, sizeof(*s->fseq) );
  s->lh = (ulong *)calloc( LH_N, sizeof(ulong) );
  s->payload = payload; s->off = off; s->sz = sz; s->n_payload = n_payload; s->rate_fps = rate_fps;
  s->device = device; s->batch_txn = batch_txn; s->max_inflight = max_inflight ? max_inflight : 2UL;
  s->zc = zero_copy;
  if( zero_copy && fdgpu_host_register( s->in_dcache, in_bytes + 128UL ) ) {
    fdgpu_mcache_delete( s->mc ); free( s->in_dcache ); free( s->frag_chunk ); free( (void *)s->fseq ); free( s->lh );
    free( s ); return -3;
  }
  pthread_mutex_init( &s->mu, NULL );
  pthread_t prod, th[64]; sb_tile_arg_t args[64];
  for( int t=0; t<tiles; t++ ) { args[t].s = s; args[t].idx = t; pthread_create( &th[t], NULL, sb_tile, &args[t] ); }
  pthread_create( &prod, NULL, sb_producer, s );
  while( atomic_load( &s->ready ) < tiles && !atomic_load( &s->fail ) ) ;
  atomic_store( &s->go, 1 );
  pthread_join( prod, NULL );
  for( int t=0; t<tiles; t++ ) pthread_join( th[t], NULL );
  int rc = atomic_load( &s->fail );
  memset( st, 0, sizeof(*st) );
  if( !rc ) {
    st->seconds = (double)( atomic_load( &s->t_last ) - s->t_start ) * 1e-9;
    st->frags = n_frags; st->sigs = atomic_load( &s->sigs ); st->published = s->metrics[4];
    st->frags_per_s = (double)n_frags / st->seconds;
    st->sigs_per_s = (double)st->sigs / st->seconds;
    ulong tot = 0UL;
    for( ulong i=0UL; i<LH_N; i++ ) tot += s->lh[i];
    st->lat_p50_us = tot ? lh_quantile( s->lh, tot, 0.50 ) * 1e-3 : 0.;
    st->lat_p99_us = tot ? lh_quantile( s->lh, tot, 0.99 ) * 1e-3 : 0.;
    st->lat_max_us = (double)s->lmax * 1e-3;
    memcpy( st->metrics, s->metrics, sizeof(st->metrics) );
    st->overruns = atomic_load( &s->overruns );
    for( int i=0; i<4; i++ ) st->tile_ns[i] = atomic_load( &s->ns[i] );
  }
  if( zero_copy ) fdgpu_host_unregister( s->in_dcache );
  fdgpu_mcache_delete( s->mc ); free( s->in_dcache ); free( s->frag_chunk ); free( (void *)s->fseq ); free( s->lh );
  pthread_mutex_destroy( &s->mu );
  free( s );
  return rc ? -rc - 10 : 0;
}
