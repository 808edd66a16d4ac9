/* ref_stem_harness.c -- TEST INFRASTRUCTURE ONLY.

   INTEGRATION.md §2's tile patch, compiled against the reference's own
   stem: src/disco/stem/fd_stem.c is #included in place with the GPU
   tile's callbacks (the way src/disco/verify/fd_verify_tile.c:253-263
   instantiates it), and its run loop STEM_(run1) drives
   libfdgpu_vtile.so over reference tango objects -- an fd_mcache /
   dcache in link, an fd_mcache out link whose reliable consumer returns
   credits through an fd_fseq, the stem's own in-link fseq and metrics
   (src/tango/{mcache,dcache,fseq}, src/disco/metrics, all compiled in
   place by oracle/Makefile with plain gcc, -z defs, no stand-ins).

   What the run exercises of the stem contract (src/disco/stem/fd_stem.c):
   - STEM_CALLBACK_BEFORE_CREDIT (:499-503): the overrun confirmation of
     the last taken frag (below) and fdgpu_vtile_housekeep;
   - STEM_CALLBACK_AFTER_CREDIT (:526-537): verdicts drained and
     published with fd_stem_publish, at most STEM_BURST per call, only
     when the out link has STEM_BURST credits (:512-523 backpressure);
   - STEM_CALLBACK_BEFORE_FRAG (:627), DURING_FRAG (:668): the tile's
     before_frag / during_frag_chunk;
   - STEM_CALLBACK_RETURNABLE_FRAG (:688-697): a frag the tile could not
     take (staging full, -2, or a copy backlog) is handed back and polled
     again;
   - the stem's overrun-while-reading check (:673-686): a frag
     during_frag took but the stem then found overwritten reaches neither
     RETURNABLE_FRAG nor AFTER_FRAG; the next BEFORE_CREDIT sees it still
     unconfirmed and marks it (fdgpu_vtile_during_frag_overrun), so it is
     never published, as the reference drops it.
   The producer thread stands in for a QUIC tile (quic_verify links are
   unreliable, src/app/fdctl/topology.c:167-169): it writes each frag's
   fd_txn_m_t record into the in dcache and publishes it with
   fd_mcache_publish, never waiting.  The consumer thread stands in for the
   dedup tile (verify_dedup is reliable, :170-172).  tests/test_gpu_stem.py
   compares what the consumer received with the reference tile's own
   decisions (oracle/_ref/libfdref_tile.so). */

#include <pthread.h>
#include <stdatomic.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "disco/stem/fd_stem.h"
#include "disco/metrics/fd_metrics.h"
#include "tango/fd_tango.h"
#include "../include/fd_verify_gpu.h"

#define HSTEM_BURST 64UL

typedef struct {
  /* the tile */
  fdgpu_vtile_t *        vt;
  fd_frag_meta_t const * in_mcache;
  ulong                  in_depth;
  ulong                  max_inflight;
  int                    retry;          /* during_frag did not take the frag: RETURNABLE_FRAG hands it back */
  int                    took;           /* during_frag took a frag the stem has not yet confirmed (overrun check) */
  int                    err;
  ulong                  n_frags, last_done;   /* last_done: the link's last frag was taken (confirmed) or filtered */
  /* accounting */
  ulong                  returned, stem_overruns, filtered, taken, published, bursts, drained;
  fdgpu_vtile_done_t     done[ HSTEM_BURST ];
  /* the tile's verdicts in after_frags order */
  ulong *                tr_seq; int * tr_res; ulong * tr_tag; ulong tr_cap, tr_cnt;
  /* out link */
  uchar const *          out_base;
} hstem_ctx_t;

static void
hstem_before_credit( hstem_ctx_t * ctx, fd_stem_context_t * stem, int * charge_busy ) {
  (void)stem;
  if( FD_UNLIKELY( ctx->took ) ) {              /* the stem skipped the frag after during_frag: overrun while reading */
    fdgpu_vtile_during_frag_overrun( ctx->vt );
    ctx->took = 0; ctx->stem_overruns++;
  }
  if( fdgpu_vtile_housekeep( ctx->vt, ctx->max_inflight ) ) *charge_busy = 1;
}

static void
hstem_after_credit( hstem_ctx_t * ctx, fd_stem_context_t * stem, int * opt_poll_in, int * charge_busy ) {
  (void)opt_poll_in;
  ulong n = fdgpu_vtile_after_frags( ctx->vt, ctx->done, HSTEM_BURST, 0 );
  if( !n ) return;
  *charge_busy = 1; ctx->bursts++; ctx->drained += n;
  ulong tspub = (ulong)fd_frag_meta_ts_comp( fd_tickcount() );
  for( ulong i=0UL; i<n; i++ ) {
    fdgpu_vtile_done_t const * d = &ctx->done[i];
    if( ctx->tr_cnt < ctx->tr_cap ) {
      ctx->tr_seq[ ctx->tr_cnt ] = d->seq; ctx->tr_res[ ctx->tr_cnt ] = d->result; ctx->tr_tag[ ctx->tr_cnt ] = d->tag;
      ctx->tr_cnt++;
    }
    if( d->result == FDGPU_VTILE_PUBLISH ) {    /* fd_verify_tile.c:149-151 */
      fd_stem_publish( stem, 0UL, 0UL, d->chunk, d->sz, 0UL, d->tsorig, tspub );
      ctx->published++;
    }
  }
}

static int
hstem_before_frag( hstem_ctx_t * ctx, ulong in_idx, ulong seq, ulong sig ) {
  int f = fdgpu_vtile_before_frag( ctx->vt, in_idx, seq, sig );
  if( f ) { ctx->filtered++; if( seq == ctx->n_frags - 1UL ) ctx->last_done = 1UL; }
  return f;
}

static void
hstem_during_frag( hstem_ctx_t * ctx, ulong in_idx, ulong seq, ulong sig, ulong chunk, ulong sz, ulong ctl ) {
  /* the frag's tsorig from its line (the stem read it just before this call and hands it to after_frag;
     the GPU tile returns it with the verdict instead) */
  ulong tsorig = (ulong)ctx->in_mcache[ fd_mcache_line_idx( seq, ctx->in_depth ) ].tsorig;
  int rc = fdgpu_vtile_during_frag_chunk( ctx->vt, in_idx, seq, sig, chunk, sz, ctl, tsorig );
  if( FD_LIKELY( !rc ) ) { ctx->took = 1; ctx->retry = 0; return; }
  if( rc == -2 || rc == FDGPU_VTILE_COPY_BACKLOG ) { ctx->retry = 1; ctx->returned++; return; }
  ctx->err = rc; ctx->retry = 0;                /* (the reference FD_LOG_ERRs: the run stops) */
}

static int
hstem_returnable_frag( hstem_ctx_t * ctx, ulong in_idx, ulong seq, ulong sig, ulong chunk, ulong sz, ulong tsorig,
                       ulong tspub, fd_stem_context_t * stem ) {
  (void)in_idx; (void)sig; (void)chunk; (void)sz; (void)tsorig; (void)tspub; (void)stem;
  if( ctx->retry ) { ctx->retry = 0; return 1; }   /* not taken: the stem polls this seq again */
  if( ctx->took ) { ctx->took = 0; ctx->taken++; }
  if( seq == ctx->n_frags - 1UL ) ctx->last_done = 1UL;
  return 0;
}

static int
hstem_should_shutdown( hstem_ctx_t * ctx ) {
  if( ctx->err ) return 1;
  return ctx->last_done && !ctx->took && !ctx->retry && !fdgpu_vtile_pending( ctx->vt );
}

#define STEM_BURST                    HSTEM_BURST
#define STEM_CALLBACK_CONTEXT_TYPE    hstem_ctx_t
#define STEM_CALLBACK_CONTEXT_ALIGN   64UL
#define STEM_CALLBACK_SHOULD_SHUTDOWN hstem_should_shutdown
#define STEM_CALLBACK_BEFORE_CREDIT   hstem_before_credit
#define STEM_CALLBACK_AFTER_CREDIT    hstem_after_credit
#define STEM_CALLBACK_BEFORE_FRAG     hstem_before_frag
#define STEM_CALLBACK_DURING_FRAG     hstem_during_frag
#define STEM_CALLBACK_RETURNABLE_FRAG hstem_returnable_frag
#include "disco/stem/fd_stem.c"

/* ---- the run ---------------------------------------------------------- */

#include "ref_stem.h"

typedef struct {
  ref_stem_cfg_t *       c;
  fd_frag_meta_t *       mcache;
  uchar *                dcache;          /* chunk 0 at dcache */
  ulong                  rec_stride, slots;
  _Atomic int            go;
} hprod_t;

static ulong hnow( void ) { struct timespec ts; clock_gettime( CLOCK_MONOTONIC, &ts ); return (ulong)ts.tv_sec*1000000000UL + (ulong)ts.tv_nsec; }

static void * hproducer( void * _a ) {
  hprod_t * a = (hprod_t *)_a;
  ref_stem_cfg_t * c = a->c;
  while( !atomic_load( &a->go ) ) FD_SPIN_PAUSE();
  ulong t0 = hnow();
  for( ulong s=0UL; s<c->n_frags; s++ ) {
    if( c->rate_fps ) { ulong due = t0 + (ulong)( (double)s * 1e9 / (double)c->rate_fps ); while( hnow() < due ) FD_SPIN_PAUSE(); }
    ulong p = s % c->n_payload;
    /* the record's dcache slot: depth + 2 slots in a ring (fd_dcache_req_data_sz's depth + burst), so the slot of
       seq s is rewritten only after line s has been republished with s + depth -- a reader that re-checks the
       line after copying (the stem, the GPU copy) never accepts a half-rewritten record */
    ulong chunk = ( s % a->slots ) * ( a->rec_stride / FD_CHUNK_SZ );
    uchar * rec = a->dcache + chunk * FD_CHUNK_SZ;
    ulong psz = c->sz[p];
    memset( rec, 0, 80UL );
    *(ushort *)( rec + 8 ) = (ushort)psz;                               /* fd_txn_m_t payload_sz */
    memcpy( rec + 80UL, c->payload + c->off[p], psz );
    ulong ts = (ulong)fd_frag_meta_ts_comp( fd_tickcount() );
    fd_mcache_publish( a->mcache, c->in_depth, s, 0UL, chunk, 80UL + psz, 0UL, ts, ts );
  }
  return NULL;
}

typedef struct {
  ref_stem_cfg_t *       c;
  fd_frag_meta_t const * mcache;
  ulong                  depth;
  ulong *                fseq;
  uchar const *          base;
  _Atomic ulong          expect;         /* published count once the stem has returned (ULONG_MAX before) */
  ulong                  consumed;
} hcons_t;

static void * hconsumer( void * _a ) {
  hcons_t * a = (hcons_t *)_a;
  ref_stem_cfg_t * c = a->c;
  ulong seq = 0UL;
  for(;;) {
    if( seq >= atomic_load( &a->expect ) ) break;
    fd_frag_meta_t const * line = a->mcache + fd_mcache_line_idx( seq, a->depth );
    ulong s0 = FD_VOLATILE_CONST( line->seq );
    if( fd_seq_lt( s0, seq ) ) { fd_fseq_update( a->fseq, seq ); FD_SPIN_PAUSE(); continue; }   /* idle: credit all */
    FD_COMPILER_MFENCE();
    ulong chunk = line->chunk, sz = line->sz;
    FD_COMPILER_MFENCE();
    if( FD_VOLATILE_CONST( line->seq ) != seq ) { a->consumed = ~0UL; return NULL; }   /* reliable: never overrun */
    uchar rec[ 2304 ];
    if( sz > sizeof(rec) ) { a->consumed = ~1UL; return NULL; }
    memcpy( rec, a->base + chunk * FD_CHUNK_SZ, sz );
    ulong pe = 80UL + *(ushort const *)( rec + 8 );
    if( ( pe & 1UL ) && pe < sz ) rec[ pe ] = 0;                       /* the alignment byte, as link_trace */
    if( seq < c->c_cap ) { c->c_hash[ seq ] = fdgpu_xxh64( 0UL, rec, sz ); c->c_sz[ seq ] = sz; }
    seq++;
    a->consumed = seq;
    if( !( seq & 15UL ) || seq >= atomic_load( &a->expect ) ) fd_fseq_update( a->fseq, seq );
    if( c->consumer_pause_every && !( seq % c->consumer_pause_every ) ) {
      fd_fseq_update( a->fseq, seq );
      ulong t = hnow(); while( hnow() - t < c->consumer_pause_ns ) FD_SPIN_PAUSE();
    }
  }
  fd_fseq_update( a->fseq, seq );
  return NULL;
}

static void * aligned( ulong align, ulong sz ) {
  void * p = NULL;
  if( posix_memalign( &p, align, ( sz + align - 1UL ) & ~( align - 1UL ) ) ) return NULL;
  memset( p, 0, sz );
  return p;
}

int
ref_stem_run( ref_stem_cfg_t * c ) {
  if( !c->n_frags || !c->n_payload || !fd_ulong_is_pow2( c->in_depth ) || !fd_ulong_is_pow2( c->out_depth ) ) return -1;
  int rc = -3;
  /* in link: mcache + a dcache of in_depth record slots (fd_dcache_req_data_sz's role: a slot per line) */
  ulong rec_stride = 1344UL;                                             /* 80 + 1232, whole 64-B chunks */
  ulong slots = c->in_depth + 2UL;
  void * in_mc_mem  = aligned( fd_mcache_align(), fd_mcache_footprint( c->in_depth, 0UL ) );
  void * out_mc_mem = aligned( fd_mcache_align(), fd_mcache_footprint( c->out_depth, 0UL ) );
  void * fseq_in_mem  = aligned( fd_fseq_align(), fd_fseq_footprint() );
  void * fseq_out_mem = aligned( fd_fseq_align(), fd_fseq_footprint() );
  ulong  in_bytes = slots * rec_stride + 4096UL;
  uchar * in_dc = (uchar *)aligned( 4096UL, in_bytes );
  void * metrics_mem = aligned( FD_METRICS_ALIGN, FD_METRICS_FOOTPRINT( 1UL, 1UL ) );
  void * scratch = aligned( FD_STEM_SCRATCH_ALIGN, stem_scratch_footprint( 1UL, 1UL, 1UL ) );
  hstem_ctx_t * ctx = (hstem_ctx_t *)aligned( 64UL, sizeof(hstem_ctx_t) );
  if( !in_mc_mem || !out_mc_mem || !fseq_in_mem || !fseq_out_mem || !in_dc || !metrics_mem || !scratch || !ctx ) goto done;

  fd_frag_meta_t * in_mc  = fd_mcache_join( fd_mcache_new( in_mc_mem,  c->in_depth,  0UL, 0UL ) );
  fd_frag_meta_t * out_mc = fd_mcache_join( fd_mcache_new( out_mc_mem, c->out_depth, 0UL, 0UL ) );
  ulong * in_fseq  = fd_fseq_join( fd_fseq_new( fseq_in_mem,  0UL ) );
  ulong * out_fseq = fd_fseq_join( fd_fseq_new( fseq_out_mem, 0UL ) );
  if( !in_mc || !out_mc || !in_fseq || !out_fseq ) goto done;
  ulong * metrics = fd_metrics_register( (ulong *)fd_metrics_new( metrics_mem, 1UL, 1UL ) );

  /* the GPU tile: its out dcache holds the out link's depth of published records plus its pending frags, which
     its staging bounds (4 slots of batch_txn per engine context, at most 2 contexts here) */
  fdgpu_vtile_opts_t o; memset( &o, 0, sizeof(o) );
  o.nctx = c->nctx;
  ctx->vt = fdgpu_vtile_new_opts( c->device, c->batch_txn, c->tcache_depth, c->seed,
                                  ( c->out_depth + 8UL * c->batch_txn + 64UL ) * 2304UL, FDGPU_SEMANTICS_AVX512, &o );
  if( !ctx->vt ) { rc = -4; goto done; }
  ulong wmark = ( slots - 1UL ) * ( rec_stride / FD_CHUNK_SZ );
  if( fdgpu_vtile_set_in( ctx->vt, 0UL, FDGPU_VTILE_IN_KIND_QUIC, in_dc, 0UL, wmark ) ) { rc = -5; goto done; }
  fdgpu_mcache_t * wrap = NULL;
  if( c->zero_copy ) {                        /* the GPU copies from the registered in dcache, re-checking the line */
    if( fdgpu_host_register( in_dc, in_bytes ) ) { rc = -6; goto done; }
    wrap = fdgpu_mcache_wrap( in_mc, c->in_depth );
    fdgpu_mcache_t const * mcs[1] = { wrap };
    if( !wrap || fdgpu_vtile_set_in_links( ctx->vt, mcs, 1 ) ) { rc = -7; goto done; }
  }
  ctx->in_mcache = in_mc; ctx->in_depth = c->in_depth; ctx->n_frags = c->n_frags;
  ctx->max_inflight = c->max_inflight ? c->max_inflight : 1UL;
  ctx->tr_seq = c->tr_seq; ctx->tr_res = c->tr_res; ctx->tr_tag = c->tr_tag; ctx->tr_cap = c->tr_cap;
  ctx->out_base = fdgpu_vtile_out_dcache( ctx->vt );

  hprod_t prod = { .c = c, .mcache = in_mc, .dcache = in_dc, .rec_stride = rec_stride, .slots = slots };
  atomic_store( &prod.go, 0 );
  hcons_t cons = { .c = c, .mcache = out_mc, .depth = c->out_depth, .fseq = out_fseq, .base = ctx->out_base, .consumed = 0UL };
  atomic_store( &cons.expect, ~0UL );
  pthread_t pt, ct;
  if( pthread_create( &pt, NULL, hproducer, &prod ) ) goto done_vt;
  if( pthread_create( &ct, NULL, hconsumer, &cons ) ) { atomic_store( &prod.go, 1 ); pthread_join( pt, NULL ); goto done_vt; }

  fd_rng_t _rng[1];
  fd_rng_t * rng = fd_rng_join( fd_rng_new( _rng, (uint)c->seed, 0UL ) );
  fd_frag_meta_t const * in_mcs[1] = { in_mc };
  ulong * in_fseqs[1] = { in_fseq };
  fd_frag_meta_t * out_mcs[1] = { out_mc };
  ulong cons_out[1] = { 0UL };
  ulong * cons_fseq[1] = { out_fseq };
  atomic_store( &prod.go, 1 );
  stem_run1( 1UL, in_mcs, in_fseqs, 1UL, out_mcs, 1UL, cons_out, cons_fseq, HSTEM_BURST, 0L, rng, scratch, ctx );
  atomic_store( &cons.expect, ctx->published );
  pthread_join( pt, NULL );
  pthread_join( ct, NULL );

  c->out[0]  = ctx->drained;       c->out[1] = cons.consumed;    c->out[2] = ctx->returned;
  c->out[3]  = ctx->stem_overruns; c->out[4] = ctx->filtered;    c->out[5] = ctx->taken;
  c->out[6]  = ctx->published;     c->out[7] = ctx->bursts;
  volatile ulong const * lin = fd_metrics_link_in( metrics, 0UL );
  c->out[8]  = lin[ FD_METRICS_COUNTER_LINK_CONSUMED_COUNT_OFF ];
  c->out[9]  = lin[ FD_METRICS_COUNTER_LINK_FILTERED_COUNT_OFF ];
  c->out[10] = lin[ FD_METRICS_COUNTER_LINK_OVERRUN_POLLING_FRAG_COUNT_OFF ];
  c->out[11] = lin[ FD_METRICS_COUNTER_LINK_OVERRUN_READING_FRAG_COUNT_OFF ];
  c->out[12] = fd_metrics_tile( metrics )[ MIDX( COUNTER, TILE, BACKPRESSURE_COUNT ) ];
  c->out[13] = ctx->tr_cnt;
  c->out[14] = (ulong)(long)ctx->err;
  fdgpu_vtile_metrics( ctx->vt, c->tile_metrics );
  rc = ctx->err ? -8 : 0;
done_vt:
  fdgpu_vtile_delete( ctx->vt );
  if( wrap ) fdgpu_mcache_delete( wrap );
  if( c->zero_copy ) fdgpu_host_unregister( in_dc );
done:
  free( in_mc_mem ); free( out_mc_mem ); free( fseq_in_mem ); free( fseq_out_mem ); free( in_dc ); free( metrics_mem );
  free( scratch ); free( ctx );
  return rc;
}
