#ifndef HEADER_fd_verify_gpu_h
#define HEADER_fd_verify_gpu_h

/* fd_verify_gpu.h -- the verify tile's frag callbacks with the GPU engine
   behind them (libfdgpu_vtile.so, host C over libfdgpu_ed25519.so).

   Replaces, for one verify tile, the work of

     before_frag   src/disco/verify/fd_verify_tile.c:36-59  (round robin)
     during_frag   src/disco/verify/fd_verify_tile.c:65-101 (copy to out dcache)
     after_frag    src/disco/verify/fd_verify_tile.c:103-157
                   (fd_txn_parse, bundle state, fd_txn_verify = HA dedup
                   + fd_ed25519_verify_batch_single_msg, publish)

   The reference does all of after_frag synchronously per frag.  Here
   during_frag hands the frag to the GPU: either it copies the frag into
   the out dcache as the reference does and the batch uploads it, or
   (zero-copy intake, fdgpu_vtile_set_in_links) the GPU itself copies it
   from the in dcache into the device and into the out-dcache record,
   re-checking the frag's in-mcache line after the copy as the stem does.
   Parse and verify happen on the device; after_frags drains verdicts in
   frag order and applies the parts of after_frag that depend on order --
   bundle state, the tcache HA dedup query / insert, metrics and the
   publish decision -- with the reference's decision order, so the
   published stream and the four metrics equal the reference tile's for
   the same input stream (tests/test_gpu_vtile.py, and at 200K frags per
   leg tests/test_gpu_stream_parity.py, against the reference tile
   compiled in place).

   Also here: a minimal tango (mcache / dcache rings with the frag
   metadata and chunk addressing of src/tango/mcache/fd_mcache.h and
   src/tango/dcache/fd_dcache.h) and a tcache with fd_tcache's
   insert/evict semantics (src/tango/tcache/fd_tcache.h:281-404), used
   by the tile and by the streaming benchmark (BASELINE configs[4]). */

#include "fd_ed25519_gpu.h"

#ifdef __cplusplus
extern "C" {
#endif

/* ---- frag record: fd_txn_m_t (src/disco/fd_txn_m_t.h:14-64) -------- */

typedef struct fdgpu_txnm {
  unsigned long  reference_slot;
  unsigned short payload_sz;
  unsigned short txn_t_sz;
  unsigned int   source_ipv4;
  unsigned char  source_tpu;
  unsigned char  _pad0[ 7 ];
  unsigned long  bundle_id;
  unsigned long  bundle_txn_cnt;
  unsigned char  commission;
  unsigned char  commission_pubkey[ 32 ];
  unsigned char  _pad1[ 7 ];
  /* followed by payload[ payload_sz ], then (after verify) the fd_txn_t
     at the next 2-byte boundary */
} fdgpu_txnm_t;

#define FDGPU_TXNM_HDR_SZ (80UL)
#define FDGPU_CHUNK_SZ    (64UL)   /* FD_CHUNK_SZ, src/tango/fd_tango_base.h */

/* ---- HA dedup tag -------------------------------------------------- */

/* fd_hash( seed, sig0, 64 ) of fd_txn_verify (fd_verify_tile.h:79):
   XXH64 of the transaction's first signature */
unsigned long fdgpu_dedup_tag( unsigned long seed, unsigned char const sig[ 64 ] );
/* XXH64 of n bytes (the link's verdict trace hashes published records with it) */
unsigned long fdgpu_xxh64( unsigned long seed, unsigned char const * p, unsigned long n );

/* ---- tcache: HA dedup of the last `depth` unique tags -------------- */

typedef struct fdgpu_tcache fdgpu_tcache_t;

fdgpu_tcache_t * fdgpu_tcache_new   ( unsigned long depth );
void             fdgpu_tcache_delete( fdgpu_tcache_t * tc );
/* 1 if tag is among the last depth unique tags inserted (tag 0 is null) */
int              fdgpu_tcache_query ( fdgpu_tcache_t const * tc, unsigned long tag );
/* FD_TCACHE_INSERT: returns 1 (dup, nothing changes) or inserts tag,
   evicting the oldest when depth tags are held, and returns 0 */
int              fdgpu_tcache_insert( fdgpu_tcache_t * tc, unsigned long tag );

/* ---- mcache / dcache ----------------------------------------------- */

typedef struct fdgpu_frag_meta {   /* fd_frag_meta_t fields the verify path uses */
  unsigned long seq;
  unsigned long sig;
  unsigned int  chunk;
  unsigned int  sz;
  unsigned long tsorig;
  unsigned long tspub;
} fdgpu_frag_meta_t;

typedef struct fdgpu_mcache fdgpu_mcache_t;

fdgpu_mcache_t * fdgpu_mcache_new    ( unsigned long depth, unsigned long seq0 );   /* depth: power of 2 */
void             fdgpu_mcache_delete ( fdgpu_mcache_t * mc );
/* producer: publish frag seq (seq must be the producer's next) */
void             fdgpu_mcache_publish( fdgpu_mcache_t * mc, unsigned long seq, unsigned long sig, unsigned int chunk,
                                       unsigned int sz, unsigned long tsorig, unsigned long tspub );
/* consumer: 0 = frag seq copied to *out; 1 = not yet published; -1 = overrun
   (the producer has lapped seq).  Lines are fd_frag_meta_t's 32 bytes: out
   tsorig / tspub are the compressed low 32 bits of the timestamps given to
   publish (fd_frag_meta_ts_comp). */
int              fdgpu_mcache_poll   ( fdgpu_mcache_t const * mc, unsigned long seq, fdgpu_frag_meta_t * out );
/* the same, plus the seq the line held (*seq_found): where an overrun consumer resumes (the stem's
   FD_MCACHE_WAIT seq_found, src/tango/mcache/fd_mcache.h:451-520; src/disco/stem/fd_stem.c:590-596) */
int              fdgpu_mcache_query  ( fdgpu_mcache_t const * mc, unsigned long seq, fdgpu_frag_meta_t * out,
                                       unsigned long * seq_found );
/* A handle on the reference's own mcache: `lines` is what fd_mcache_join returns (an fd_frag_meta_t
   array of depth lines, src/tango/mcache/fd_mcache.h:113,137; 32-byte lines laid out as
   src/tango/fd_tango_base.h:146-203; line of seq = seq & (depth-1), FD_MCACHE_LG_INTERLEAVE 0).  Nothing
   is copied or written; the producer keeps publishing with fd_mcache_publish.  fdgpu_mcache_delete
   frees only the handle (and unregisters the lines' pages if fdgpu_vtile_set_in_links registered them).
   NULL if depth is not a power of 2 or lines is not 32-byte aligned. */
fdgpu_mcache_t * fdgpu_mcache_wrap   ( void * lines, unsigned long depth );
unsigned long    fdgpu_mcache_depth  ( fdgpu_mcache_t const * mc );
void *           fdgpu_mcache_lines  ( fdgpu_mcache_t * mc );

/* next chunk after a frag of sz bytes at chunk, wrapping to chunk0 past
   wmark (fd_dcache_compact_next, src/tango/dcache/fd_dcache.h) */
unsigned long    fdgpu_dcache_compact_next( unsigned long chunk, unsigned long sz, unsigned long chunk0,
                                            unsigned long wmark );

/* ---- the GPU verify tile ------------------------------------------ */

#define FDGPU_VTILE_PUBLISH          (0)
#define FDGPU_VTILE_PARSE_FAIL       (1)
#define FDGPU_VTILE_VERIFY_FAIL      (2)
#define FDGPU_VTILE_DEDUP_FAIL       (3)
#define FDGPU_VTILE_BUNDLE_PEER_FAIL (4)
#define FDGPU_VTILE_OVERRUN          (5)   /* zero-copy intake: the producer reused the frag's line while the GPU copied it */
#define FDGPU_VTILE_GPU_FAULT        (6)   /* the frag's GPU batch failed: no verdict, never published (the
                                              reference tile would FD_LOG_ERR, fd_verify_tile.c:74-84) */

typedef struct fdgpu_vtile_done {
  unsigned long seq;      /* the frag's seq on its in link, as given to during_frag (full 64 bits) */
  unsigned long tsorig;
  unsigned long chunk;    /* out dcache chunk of the fd_txn_m_t record */
  unsigned long sz;       /* realized footprint (fd_txn_m_realized_footprint) when published */
  unsigned long tag;      /* HA dedup tag (0 for bundles) */
  int           result;   /* FDGPU_VTILE_* */
  int           code;     /* the GPU's code for the txn: FD_ED25519_* (0, -1, -2, -3), FDGPU_ERR_PARSE / _OVERRUN;
                             0 for a GPU fault */
  unsigned long in_idx;   /* the in link, as given to during_frag (the stem's in_idx) */
  /* diagnostics of the GPU batch that verified the frag (a verdict can be traced to its batch) */
  unsigned int  ctx;      /* the tile's engine context */
  unsigned int  batch_txns;   /* transactions in the batch */
  unsigned int  batch_pos;    /* the frag's position in it */
  int           path;     /* the batch's engine path: FDGPU_PATH_* */
} fdgpu_vtile_done_t;

typedef struct fdgpu_vtile fdgpu_vtile_t;

/* GPU-side metrics of a tile (batches submitted, in-flight
   depth, GPU verify latency histogram; plus overruns and faults), next to
   the reference's verify counters of fdgpu_vtile_metrics. */
#define FDGPU_VTILE_LAT_BUCKETS ((unsigned long)FDGPU_LAT_BUCKETS)
typedef struct fdgpu_vtile_gpu_metrics {
  unsigned long batches;          /* batches launched */
  unsigned long batch_txns;       /* transactions in them (batches / batch_txns = mean batch) */
  unsigned long inflight;         /* launched batches not yet drained, now */
  unsigned long inflight_max;     /* high-water mark of inflight */
  unsigned long pending;          /* frags between during_frag and after_frags, now */
  unsigned long overruns;         /* frags returned as FDGPU_VTILE_OVERRUN */
  unsigned long gpu_fault_frags;  /* frags returned as FDGPU_VTILE_GPU_FAULT */
  unsigned long faults;           /* engine contexts seen faulted */
  unsigned long lat_hist[ FDGPU_VTILE_LAT_BUCKETS ];  /* per batch, launch -> verdicts polled, summed over the
                                                         tile's engine contexts (buckets: fdgpu_lat_bucket) */
  unsigned long wait_ns;          /* host time after_frags spent blocked on a batch not yet complete */
  unsigned long poll_ns;          /* ... in non-blocking completion polls (fdgpu_ed25519_poll_raw) */
  unsigned long after_ns;         /* ... in after_frag proper (dedup, overrun check, publish) */
  unsigned long launch_ns;        /* host time inside batch launches and early copies (in during_frag, housekeep or a drain) */
  unsigned long copies;           /* zero-copy: early GPU copies started (housekeep, fdgpu_vtile_copy) */
  unsigned long copy_lat_n, copy_lat_ns_sum, copy_lat_ns_max;   /* ... of them timed: launch -> completion seen */
  unsigned long gather_gpu[ 8 ];  /* every GPU copy (early or at a batch launch), on the GPU clock, summed over the
                                     tile's contexts: fdgpu_ed25519_gather_stats (count, launch -> start sum / max,
                                     start -> end sum / max, issue -> start sum / max, ns, issue -> start over 250 us) */
  unsigned long phase[ 9 ];       /* fdgpu_ed25519_phase_stats summed over the tile's contexts (maxima: max) */
  unsigned long copy_backlog;     /* during_frag calls refused with FDGPU_VTILE_COPY_BACKLOG */
  unsigned long launcher[ 6 ];    /* the tile's launch thread (opts.launcher), fdgpu_launcher_stats: commands issued,
                                     ns issuing them, deepest queue, pushes that waited for room, longest command (ns),
                                     commands over 250 us (0s without one) */
  unsigned long host_copy[ 4 ];   /* the tile's copy threads (opts.copy_threads): records copied, ns copying (summed over
                                     threads), records found overrun after their copy, ns the tile waited for a copy */
} fdgpu_vtile_gpu_metrics_t;

/* device: HIP device; batch_txn: transactions per GPU batch (staging
   slot); tcache_depth: HA dedup depth (verify.tcache_depth); seed: the
   dedup hash seed (ctx->hashmap_seed); out_dcache_bytes: size of the
   tile's out dcache (fd_txn_m_t records, 64-B chunks);  semantics:
   FDGPU_SEMANTICS_*.  NULL on failure (fdgpu_last_error).  Tuning comes
   only through fdgpu_vtile_opts_t (fdgpu_vtile_new: every field 0 =
   default); nothing is read from the environment. */
#define FDGPU_VTILE_COPY_WAIT_NS (50000UL)   /* default copy_wait_ns */
#define FDGPU_VTILE_COPY_MIN     (4096UL)    /* default copy_min */
#define FDGPU_VTILE_MAX_UNCOPIED (16384UL)   /* default max_uncopied */
/* during_frag's answer when max_uncopied frags await their GPU copy: the frag was not taken.  The copies
   of the frags taken have been started; poll them (fdgpu_vtile_housekeep or fdgpu_vtile_copy) and retry
   later.  A tile that takes frags faster than the GPU copies them thus falls behind in the link, where
   a lapping producer overruns it at the mcache poll (frags lost, as for a slow reference tile), instead
   of taking frags whose copy would start after the producer reused their line (overrun at copy time). */
#define FDGPU_VTILE_COPY_BACKLOG (-5)
typedef struct fdgpu_vtile_opts {
  int           nctx;            /* engine contexts per tile, 1..3 (0 = 2): batches of consecutive frags go to them in
                                    turn, launched staggered, so a frag does not wait for a whole running batch */
  int           host_dedup_tag;  /* 1: after_frag computes the HA dedup tag on the host (reads the payload; A/B only) */
  unsigned long small_max;       /* batches of at most this many signatures take the engine's latency path
                                    (0 = half the batch limit, at most the engine default) */
  unsigned long min_batch;       /* housekeep: a partial batch below this many frags waits ... (0 = never waits) */
  unsigned long max_wait_ns;     /* ... until its oldest frag has waited this long (0 = 2 ms) */
  unsigned long copy_wait_ns;    /* zero-copy: housekeep starts the GPU copy of the frags taken since the last one
                                    once the oldest has waited this long (0 = FDGPU_VTILE_COPY_WAIT_NS) ... */
  unsigned long copy_min;        /* ... or once this many are waiting (0 = FDGPU_VTILE_COPY_MIN) */
  unsigned int  gather_cus;      /* CUs of the GPU reserved for the copies (fdgpu_ed25519_reserve_gather_cus; 0 = none) */
  unsigned long max_uncopied;    /* zero-copy: frags taken whose copy has not completed, at most (0 =
                                    FDGPU_VTILE_MAX_UNCOPIED); at the bound during_frag returns FDGPU_VTILE_COPY_BACKLOG */
  int           cu_split;        /* 1 (with gather_cus): context k's verify kernels run on the k-th of nctx disjoint
                                    shares of the other CUs (fdgpu_ed25519_reserve_cus), so the staggered batches
                                    of one tile do not share SIMDs; 0: every context on all of them */
  int           cu_exclusive;    /* each context's latency-path workgroups alone on their CU
                                    (fdgpu_ed25519_set_cu_exclusive): 0 = default (on: paced p99 at 10M frags/s
                                    0.96 vs 1.06 ms, knee 10M vs 7.5M, profiles/r04/q); -1 = off; 1..4 explicit */
  int           launcher;        /* 1: the tile's contexts make their batch launches and copies on a launch thread
                                    of the tile's own (fdgpu_launcher_new): the tile's thread only queues them;
                                    0: on the tile's thread */
  int           launcher_core;   /* with launcher: 1 + the CPU its thread is pinned to (0: not pinned) */
  int           copy_threads;    /* zero-copy intake: 0 = the GPU copy writes each record into the out dcache as it
                                    reads it (the record crosses PCIe twice); 1..FDGPU_VTILE_COPY_THREADS_MAX = that
                                    many host threads of the tile copy the records in -> out dcache instead (as the
                                    reference's during_frag does, fd_verify_tile.c:96-101), re-checking each frag's
                                    mcache line after the copy, and the GPU only reads them */
  int           copy_cores[ 8 ]; /* with copy_threads: 1 + the CPU copy thread i is pinned to (0: not pinned) */
  int           lat_share;       /* with cu_exclusive: each context's latency-path walk fits 1/lat_share of the CUs
                                    left by the gathers (fdgpu_ed25519_set_lat_share): 0 = default (1/nctx);
                                    -1 = no limit (a walk may be wider than its share: A/B only) */
} fdgpu_vtile_opts_t;
#define FDGPU_VTILE_COPY_THREADS_MAX 8

fdgpu_vtile_t * fdgpu_vtile_new( int device, unsigned long batch_txn, unsigned long tcache_depth, unsigned long seed,
                                 unsigned long out_dcache_bytes, int semantics );
fdgpu_vtile_t * fdgpu_vtile_new_opts( int device, unsigned long batch_txn, unsigned long tcache_depth,
                                      unsigned long seed, unsigned long out_dcache_bytes, int semantics,
                                      fdgpu_vtile_opts_t const * opts );
void            fdgpu_vtile_delete( fdgpu_vtile_t * vt );
unsigned char * fdgpu_vtile_out_dcache( fdgpu_vtile_t * vt );   /* chunk c is at base + 64 c */

/* The stem's callbacks (src/disco/stem/fd_stem.c:627,668,700) take the in link as in_idx and the frag's
   full 64-bit seq on that link; so do these.  fdgpu_vtile_set_in records what the reference tile keeps
   per in link (ctx->in_kind[ in_idx ], ctx->in[ in_idx ].mem / chunk0 / wmark, fd_verify_tile.c:181-
   230): its kind (FDGPU_VTILE_IN_KIND_*; a link never set is QUIC) and its data region -- chunk c of
   the link is at mem + 64 c (fd_chunk_to_laddr), valid for chunk0 <= c <= wmark.  The region must hold
   an MTU of readable bytes from every chunk up to wmark (as a dcache sized by fd_dcache_req_data_sz
   does): FDGPU_TPU_RAW_MTU for QUIC / bundle / send links, FDGPU_GOSSIP_MSG_MAX for a gossip link (the
   2048-byte frames fd_verify_tile.c:89-90 accepts).  Call while no frag is pending; 0, or -1 for a bad
   in_idx / kind. */
int             fdgpu_vtile_set_in( fdgpu_vtile_t * vt, unsigned long in_idx, int in_kind, void const * mem,
                                    unsigned long chunk0, unsigned long wmark );
/* STEM_CALLBACK_DURING_FRAG( ctx, in_idx, seq, sig, chunk, sz, ctl ) (fd_verify_tile.c:65-101), plus the
   frag's tsorig (the stem hands it to after_frag; here after_frags returns it): the frag at chunk of
   in link in_idx.  A chunk outside [chunk0, wmark] is -4 (the reference's FD_LOG_ERR).  Otherwise as
   fdgpu_vtile_during_frag. */
int             fdgpu_vtile_during_frag_chunk( fdgpu_vtile_t * vt, unsigned long in_idx, unsigned long seq,
                                               unsigned long sig, unsigned long chunk, unsigned long sz,
                                               unsigned long ctl, unsigned long tsorig );
/* during_frag of the frag at `frag` (sz bytes) from in link in_idx.  QUIC / bundle / send links carry
   fd_txn_m_t records: the record is copied into the out dcache (or, zero-copy intake, the GPU copies
   it) and its payload submitted; sz > FDGPU_TPU_RAW_MTU or a payload past the frag or past 1232 bytes is
   -4 (the reference's FD_LOG_ERR; fdgpu_vtile_during_frag_chunk takes a payload past sz, which a lapped
   read of a header being rewritten can show, and leaves it to the overrun checks, as the reference).  A gossip link's frag is an fd_gossip_update_message_t whose vote
   transaction becomes a fresh out-dcache record (payload_sz, bundle id 0, payload), copied by the host
   as the reference does (sz > 2048 or a vote txn_sz past 1232: -4).  Only the frame's sz bytes are read
   here: a vote whose txn_sz reaches past the frame is -4.  (The reference reads vote.txn_sz bytes even
   past the frame -- the 1297-byte FD_GOSSIP_UPDATE_SZ_VOTE frame holds 1225 of them -- because its
   dcache continues there: fdgpu_vtile_during_frag_chunk does the same.)  Returns 0, or -2 when
   the out dcache or the GPU staging is full (call fdgpu_vtile_after_frags and retry), <= -3 on error. */
int             fdgpu_vtile_during_frag( fdgpu_vtile_t * vt, unsigned long in_idx, void const * frag, unsigned long sz,
                                         unsigned long seq, unsigned long tsorig );
/* Zero-copy intake: from now on during_frag leaves the frag where it
   is -- frag must then lie in a range registered with
   fdgpu_host_register (the in dcache), 16-B aligned -- and the GPU
   copies it into the out dcache record itself
   (fdgpu_ed25519_submit_raw_gather_chk): the stem's during_frag copy,
   done by the GPU shortly after during_frag (housekeep starts the copies,
   see fdgpu_vtile_opts_t.copy_wait_ns; fdgpu_vtile_copy starts them now).
   in_mc (may be NULL): the in link's mcache (its lines are registered
   with the GPU here if they are not yet); right after copying a frag the
   GPU re-reads its line, and a frag whose line the producer reused while
   it was being copied is reported FDGPU_VTILE_OVERRUN instead of
   published -- the stem's overrun check, at the same point
   (src/disco/stem/fd_stem.c:667-686).  A lap after the copy changes
   nothing.  A reliable producer must not reuse a frag's dcache bytes
   before its copy has completed (fdgpu_vtile_copy_state).  Call while no
   frag is pending; 0 on success. */
int             fdgpu_vtile_set_in_link( fdgpu_vtile_t * vt, fdgpu_mcache_t const * in_mc );
/* The same for a tile that reads n in links (the reference's verify tile
   reads every QUIC tile's link, topology.c:167-169): a frag handed to
   during_frag from in link in_idx is checked against in_mc[ in_idx ]
   (entries may be NULL; fdgpu_mcache_wrap makes one of the reference's
   own mcache).  n <= FDGPU_VTILE_IN_MAX. */
#define FDGPU_VTILE_IN_MAX   16
int             fdgpu_vtile_set_in_links( fdgpu_vtile_t * vt, fdgpu_mcache_t const * const * in_mc, int n );
/* seq of the oldest frag not yet returned by after_frags, as handed to
   during_frag, and (in_idx, may be NULL) its in link; ~0UL (both) if none */
unsigned long   fdgpu_vtile_oldest_pending_seq( fdgpu_vtile_t const * vt, unsigned long * in_idx );
/* Zero-copy intake: start the GPU copy of every frag taken and not yet
   copied; blocking: wait until every copy has completed.  0, or < 0 if a
   context failed (its frags come back as FDGPU_VTILE_GPU_FAULT). */
int             fdgpu_vtile_copy( fdgpu_vtile_t * vt, int blocking );
/* Zero-copy intake, per in link: the number of frags taken whose copy is
   not known to have completed, and (copied_next) 1 + the seq of the
   link's last frag known copied (0 if none).  While the count is nonzero
   the producer must not reuse seqs >= copied_next (a reliable link's
   credit).  Progress is picked up by housekeep, copy and after_frags. */
unsigned long   fdgpu_vtile_copy_state( fdgpu_vtile_t const * vt, int link, unsigned long * copied_next );
/* frags dropped as FDGPU_VTILE_OVERRUN */
unsigned long   fdgpu_vtile_overruns( fdgpu_vtile_t const * vt );
/* The stem's seq re-check after during_frag's HOST copy (no zero-copy
   intake) found the frag overrun: it is abandoned -- completed as
   FDGPU_VTILE_OVERRUN, never published (fd_stem.c:667-686 skips
   after_frag).  Call right after the during_frag that took it.  0, or -1
   if nothing is pending. */
int             fdgpu_vtile_during_frag_overrun( fdgpu_vtile_t * vt );

/* ---- the reference's in kinds (fd_verify_tile.c:7-10, 36-101) -------- */
#define FDGPU_VTILE_IN_KIND_QUIC     (0)
#define FDGPU_VTILE_IN_KIND_BUNDLE   (1)
#define FDGPU_VTILE_IN_KIND_GOSSIP   (2)
#define FDGPU_VTILE_IN_KIND_SEND     (3)
#define FDGPU_TPU_RAW_MTU            (1312UL)  /* FD_TPU_RAW_MTU: fd_txn_m_t header + FD_TPU_MTU, src/disco/fd_txn_m_t.h */
#define FDGPU_GOSSIP_UPDATE_TAG_VOTE (3UL)     /* src/flamenco/gossip/fd_gossip_types.h:26 */
/* what the tile reads of an fd_gossip_update_message_t (fd_gossip_types.h:128-205, x86-64 layout):
   the ulong vote.txn_sz and the vote.txn bytes */
#define FDGPU_GOSSIP_VOTE_TXN_SZ_OFF (64UL)
#define FDGPU_GOSSIP_VOTE_TXN_OFF    (72UL)
#define FDGPU_GOSSIP_MSG_MAX         (2048UL)  /* fd_verify_tile.c:89-90 */
/* before_frag's round robin: this tile is verify:idx of cnt */
void            fdgpu_vtile_set_round_robin( fdgpu_vtile_t * vt, unsigned long idx, unsigned long cnt );
/* STEM_CALLBACK_BEFORE_FRAG( ctx, in_idx, seq, sig ) (fd_verify_tile.c:36-59): 1 = this tile skips the
   frag.  By in_idx's kind (fdgpu_vtile_set_in): a QUIC frag or a bundle-tile packet (sig 0) round robin
   on the full seq; a bundle (sig != 0) only verify:0; a gossip update round robin and only a vote (sig ==
   FDGPU_GOSSIP_UPDATE_TAG_VOTE); a send-tile frag never skipped.  in_idx >= FDGPU_VTILE_IN_MAX: 1. */
int             fdgpu_vtile_before_frag( fdgpu_vtile_t const * vt, unsigned long in_idx, unsigned long seq,
                                         unsigned long sig );

/* launch the partially filled batches (call when the input is idle) */
int             fdgpu_vtile_flush( fdgpu_vtile_t * vt );
/* transactions waiting in unlaunched batches, and launched batches not yet
   drained, summed over the tile's engine contexts (fdgpu_vtile_opts_t.nctx,
   1..3, default 2: batches of consecutive frags go to the contexts in
   turn, launched staggered by a fraction of the batch duration so a frag
   does not wait for a whole running batch before its own starts) */
void            fdgpu_vtile_pipeline_state( fdgpu_vtile_t const * vt, unsigned long * filling,
                                            unsigned long * inflight );
/* adaptive batching, for the tile's housekeeping / before_credit hook:
   launch the filling batch when fewer than max_inflight batches are on
   the GPU -- batches stay small (low latency) while the GPU keeps up and
   grow with the backlog when it does not (max_inflight is capped at one
   less than the engine's 4 staging slots).  Returns 1 if it launched. */
int             fdgpu_vtile_housekeep( fdgpu_vtile_t * vt, unsigned long max_inflight );
/* after_frag for completed frags, in during_frag order: at most max
   records to out[]; blocking waits for the oldest batch (never for a
   faulted one).  Out-dcache records are reused once after_frags has
   returned them and the ring wraps: as in the reference stem, the caller
   publishes only within its out-link credits and must not call
   during_frag while a reliable consumer still lags a full out-dcache ring
   behind (the ring holds fdgpu_vtile_pending()-bounded frags; size it to
   the consumers' depth). */
unsigned long   fdgpu_vtile_after_frags( fdgpu_vtile_t * vt, fdgpu_vtile_done_t * out, unsigned long max, int blocking );
/* frags submitted but not yet returned by after_frags */
unsigned long   fdgpu_vtile_pending( fdgpu_vtile_t const * vt );
/* Fault path.  When a batch fails on the device its engine context stops:
   after_frags never blocks on it and returns each of its pending frags, in
   frag order, as FDGPU_VTILE_GPU_FAULT; during_frag moves on to the tile's
   other contexts (-3 once none is left).  fdgpu_vtile_faulted counts the
   faulted contexts; fdgpu_vtile_recover recreates them once after_frags
   has returned all their frags (0; -1 while some are pending, -2 if a new
   context could not be created).  A stem integration either treats a
   nonzero fdgpu_vtile_faulted as the reference's FD_LOG_ERR or recovers. */
int             fdgpu_vtile_faulted( fdgpu_vtile_t const * vt );
int             fdgpu_vtile_recover( fdgpu_vtile_t * vt );
/* host-side test hook: engine context k of the tile fails (fdgpu_ed25519_debug_fault); a served tile asks its
   service, which honours it only when made with fdgpu_vsvc_cfg_t.debug_hooks */
void            fdgpu_vtile_debug_fault( fdgpu_vtile_t * vt, int k );
/* host-side test hook: the launch thread (fdgpu_vtile_opts_t.launcher) fails every batch launch of engine
   context k from now on (fdgpu_ed25519_debug_fail_launch): the context faults asynchronously, on that thread */
void            fdgpu_vtile_debug_fail_launch( fdgpu_vtile_t * vt, int k );
void            fdgpu_vtile_gpu_metrics( fdgpu_vtile_t * vt, fdgpu_vtile_gpu_metrics_t * out );
/* metrics: [0] parse_fail [1] verify_fail [2] dedup_fail
   [3] bundle_peer_fail [4] published (fd_verify_tile.c:29-34) */
void            fdgpu_vtile_metrics( fdgpu_vtile_t const * vt, unsigned long out[ 5 ] );

/* ---- the verify service: several verify-tile processes on one GPU -------

   The reference runs each verify tile as a sandboxed process of its own, six by default
   (src/disco/topo/fd_topo_run.c:66-153, src/app/fdctl/config/default.toml:788).  Tile processes that
   each open a HIP context of their own contend for the GPU's queues and CUs as strangers: their batch
   chains collide (profiles/r05/n2b: two such processes per GPU lowered the paced knee from 10M to 4M
   frags/s per device).  The verify service is one process per GPU that owns the GPU: it maps the tiles'
   in links and out dcaches, takes the frags of all of its tiles from shared-memory request rings, batches
   them together (one batch holds frags of several tiles; each record still goes back into its own tile's
   out dcache and its HA dedup tag is computed with its tile's seed) and returns every verdict into its
   tile's completion ring, in the tile's order.  A tile then makes no GPU runtime call at all: its
   during_frag writes a 32-byte request, its after_frags reads 32-byte completions and does the
   order-dependent half of after_frag itself, exactly as with engine contexts of its own (same
   fdgpu_vtile_* calls, same published stream).  Precedent: WireDancer's request / response rings
   (src/wiredancer/c/wd_f1.h:71-113).

   The service's shared segment: a header, per tile a request ring, a completion ring and the tile's out
   dcache.  The service process creates it (fdgpu_vsvc_new: a file at `path`, or anonymous shared memory
   inherited by tile processes forked before fdgpu_vsvc_start), names the in regions it will map
   (fdgpu_vsvc_add_region: the in links' dcaches and mcaches, each a region id), then
   fdgpu_vsvc_start( device ) -- from here on it is the only process with a GPU context -- and calls
   fdgpu_vsvc_poll in its loop.  A tile process joins (fdgpu_vsvc_join, or the inherited handle),
   creates its tile with fdgpu_vtile_new_svc( svc, client ), tells it where the same regions lie in its
   own address space (fdgpu_vtile_set_svc_region) and uses it as any tile. */
#define FDGPU_VSVC_CLIENT_MAX 16
#define FDGPU_VSVC_RGN_MAX    16
typedef struct fdgpu_vsvc fdgpu_vsvc_t;
typedef struct fdgpu_vsvc_cfg {
  int           clients;          /* verify tiles served, 1..FDGPU_VSVC_CLIENT_MAX */
  unsigned long out_dcache_bytes; /* each tile's out dcache (fd_txn_m_t records, 64-B chunks) */
  unsigned long batch_txn;        /* transactions per GPU batch */
  unsigned long max_inflight;     /* adaptive batching: launch the filling batch while fewer than this many are on the
                                     GPU (1..3; 0 = 2), as fdgpu_vtile_housekeep */
  int           semantics;        /* FDGPU_SEMANTICS_* */
  /* the service's engine contexts, as a tile's (fdgpu_vtile_opts_t; 0 = the same defaults) */
  int           nctx;
  unsigned long small_max, min_batch, max_wait_ns, copy_wait_ns, copy_min;
  unsigned int  gather_cus;
  int           cu_split, cu_exclusive, lat_share;
  int           launcher;         /* 1: the batch launches and copies on a launch thread of the service's own */
  int           launcher_core;    /* with launcher: 1 + its CPU (0: not pinned) */
  int           debug_hooks;      /* 1: honour a tile's fdgpu_vtile_debug_fault (tests only; 0: a tile cannot fault the
                                     service's engine contexts) */
} fdgpu_vsvc_cfg_t;

/* metrics of a service, as a tile's GPU metrics: batches, transactions batched, in-flight
   high-water, latency histogram, gathers, phases, launch thread; plus frags taken / completed, passes
   of the loop that did some work, and engine contexts faulted */
typedef struct fdgpu_vsvc_stats {
  fdgpu_vtile_gpu_metrics_t gm;
  unsigned long taken, completed, fault_completions, busy_polls, polls, faults, recovered;
  unsigned long mixed_batches;      /* batches that held the frags of more than one tile */
  unsigned long loop_ns, busy_ns;   /* fdgpu_vsvc_poll time in all passes / in the passes that did work */
} fdgpu_vsvc_stats_t;

/* create the segment (no GPU call): path NULL = anonymous shared memory (for tile processes forked from
   this one).  NULL on failure. */
fdgpu_vsvc_t *  fdgpu_vsvc_new( char const * path, fdgpu_vsvc_cfg_t const * cfg );
/* a tile process: map the service segment at path (waiting up to timeout_s for it to appear) */
fdgpu_vsvc_t *  fdgpu_vsvc_join( char const * path, double timeout_s );
/* service: region id (0..FDGPU_VSVC_RGN_MAX-1) is [base, base+sz) in this process (an in link's dcache or
   mcache lines); registered with the GPU by fdgpu_vsvc_start.  Before start; 0 or -1. */
int             fdgpu_vsvc_add_region( fdgpu_vsvc_t * svc, int id, void * base, unsigned long sz );
/* service: the GPU side -- engine contexts on device, the regions and out dcaches registered -- then the
   segment reads ready (tiles may take frags before: their requests wait).  0 or < 0. */
int             fdgpu_vsvc_start( fdgpu_vsvc_t * svc, int device );
/* 1 once the service is started, -1 if its start failed, 0 before */
int             fdgpu_vsvc_ready( fdgpu_vsvc_t const * svc );
/* service: one pass of its loop (take requests, launch, copy, drain verdicts into the tiles' rings,
   recreate faulted contexts once drained); returns 1 if it did any work */
int             fdgpu_vsvc_poll( fdgpu_vsvc_t * svc );
/* service: poll until fdgpu_vsvc_stop (any process); returns 0 */
int             fdgpu_vsvc_run( fdgpu_vsvc_t * svc );
void            fdgpu_vsvc_stop( fdgpu_vsvc_t * svc );
/* frags taken from the tiles and not yet returned to them */
unsigned long   fdgpu_vsvc_pending( fdgpu_vsvc_t const * svc );
void            fdgpu_vsvc_stats( fdgpu_vsvc_t * svc, fdgpu_vsvc_stats_t * out );
/* unmap (the service also deletes its contexts and unregisters its regions; the creator of a path
   unlinks it) */
void            fdgpu_vsvc_delete( fdgpu_vsvc_t * svc );

/* test hook (no GPU call): a CPU stand-in for the GPU side of a service not started -- completes every request
   published so far with codes[ request index % ncodes ], footprint fp, the record copied into the tile's out
   dcache after the overrun check, and the HA dedup tag of its first signature; returns how many */
unsigned long   fdgpu_vsvc_debug_serve( fdgpu_vsvc_t * svc, int const * codes, unsigned long ncodes, unsigned long fp );

/* a verify tile served by svc as client (0..clients-1): no GPU call here or later.  Its out dcache is
   the segment's (fdgpu_vtile_out_dcache).  opts: the tile's own options (copy backlog, copy threads,
   host dedup tag); the GPU-side ones are the service's.  NULL on failure. */
fdgpu_vtile_t * fdgpu_vtile_new_svc( fdgpu_vsvc_t * svc, int client, unsigned long tcache_depth, unsigned long seed,
                                     fdgpu_vtile_opts_t const * opts );
/* served tile: region id lies at [base, base+sz) in this process (the same region the service added) */
int             fdgpu_vtile_set_svc_region( fdgpu_vtile_t * vt, int id, void const * base, unsigned long sz );

/* NUMA node of HIP device `device` from sysfs alone (no GPU call, so a process may ask before it forks
   its tile processes): the device-th GPU node of the KFD topology (sysfs_root/class/kfd/kfd/topology/nodes,
   nodes with SIMDs, after ROCR_VISIBLE_DEVICES and then HIP_VISIBLE_DEVICES / CUDA_VISIBLE_DEVICES), whose
   PCI function's numa_node it reads (sysfs_root/bus/pci/devices/...).  sysfs_root NULL = "/sys".  -1 if
   unknown.  Agrees with fdgpu_device_numa_node (tests/test_gpu_vsvc.py). */
int             fdgpu_gpu_numa_node_sysfs( char const * sysfs_root, int device );

/* ---- the configs[4] stream (BASELINE configs[4]) ------------------- */

typedef struct fdgpu_stream_cfg {
  unsigned long n_frags;         /* frags the producer publishes (seq 0 .. n_frags-1) */
  unsigned long batch_txn;       /* transactions per GPU batch of a tile */
  unsigned long max_inflight;    /* fdgpu_vtile_housekeep( max_inflight ) */
  double        rate_fps;        /* producer pacing, frags/s (0 = as fast as it can) */
  int           tiles;           /* T verify tiles: tile i takes seq % T == i (fd_verify_tile.c:47-48) */
  int           gpus;            /* G: tile i drives GPU i % G, run by process i % G (one process per GPU) */
  int           zero_copy;       /* tiles leave frags in the in dcache, the GPU gathers them */
  int           reliable;        /* 1: credit-based link (the producer waits for the slowest tile);
                                    0: unreliable, as the reference's quic_verify link (topology.c:167-170):
                                    the producer never waits, a lagging tile is overrun and skips frags */
  int           producers;       /* Q producer links (the reference's QUIC tiles, 0 = 1): producer q publishes
                                    about n_frags / Q frags on its own mcache, every tile reads every link with
                                    seq % T == i on each (topology.c:167-169); producer q runs in process q % G */
  int           nctx;            /* engine contexts per tile (fdgpu_vtile_opts_t.nctx; 0 = its default) */
  int           prof;            /* 1: rdtsc section profile of the tile loop (fdgpu_stream_stats_t.prof_ns) */
  unsigned long out_mult;        /* out dcache per tile, in batch limits (0 = 6) */
  unsigned long copy_wait_ns;    /* zero-copy: fdgpu_vtile_opts_t.copy_wait_ns (0 = its default) */
  unsigned long copy_min;        /* zero-copy: fdgpu_vtile_opts_t.copy_min (0 = its default) */
  unsigned int  gather_cus;      /* fdgpu_vtile_opts_t.gather_cus */
  unsigned long max_uncopied;    /* fdgpu_vtile_opts_t.max_uncopied (0 = its default) */
  int           pf_dist;         /* tile loop prefetch distance, in own frags: the mcache line pf_dist ahead and
                                    the record header of the frag pf_dist/2 ahead (0 = 1: the next own frag's
                                    line and header; 4 and 8 measured the same, profiles/r03/prep_pf_ab) */
  int           cu_split;        /* fdgpu_vtile_opts_t.cu_split of every tile */
  int           cu_exclusive;    /* fdgpu_vtile_opts_t.cu_exclusive of every tile */
  int           no_huge_pages;   /* 1: the link region in 4 KiB pages (A/B); 0: 2 MiB transparent huge pages where the
                                    kernel allows them (madvise), as the reference's workspaces use huge pages (max rate
                                    +4 %, profiles/r04/i) */
  int           launcher;        /* 1: every tile with a launch thread of its own (fdgpu_vtile_opts_t.launcher),
                                    pinned to a core of its own next to the tiles' */
  int           copy_threads;    /* fdgpu_vtile_opts_t.copy_threads of every tile, each thread on a core of its own */
  unsigned long min_batch;       /* fdgpu_vtile_opts_t.min_batch of every tile (0: none; the max-rate legs: batches
                                    above the latency path's limit, so they take the throughput path) */
  unsigned long small_max;       /* fdgpu_vtile_opts_t.small_max of every tile (0: its default, half the batch limit) */
  unsigned long hk_ns;           /* the tile loop's housekeeping (launch decision, copies, verdict poll) at most every
                                    hk_ns while frags flow (0 = 10 us) */
  int           lat_share;       /* fdgpu_vtile_opts_t.lat_share of every tile */
  int           svc;             /* 1: every tile is a process of its own, with no GPU context, served by one verify
                                    service process per GPU (fdgpu_vsvc_*) that batches the frags of all of that GPU's
                                    tiles together; 0: the tiles are threads of one process per GPU, each with its own
                                    engine contexts.  Needs a shared link (a path): the tile processes join it */
  unsigned long trace_cap;       /* > 0: every tile records up to this many verdicts in the link itself (fdgpu_link_trace,
                                    from any process; served tiles need it), instead of fdgpu_link_set_trace's arrays */
  int           prod_node[ 16 ]; /* 1 + the NUMA node producer q's mcache and in dcache part live on, and its thread runs
                                    on (0: the link's creator decides, and the producer runs by the tiles) -- the
                                    reference gives every workspace a node (src/disco/topo/fd_topob.c:505-540) */
} fdgpu_stream_cfg_t;

typedef struct fdgpu_stream_stats {
  double        seconds;         /* first frag published by the producer -> last verdict */
  unsigned long frags, sigs, published;
  double        frags_per_s, sigs_per_s;  /* verdicts / s and verified signatures / s */
  double        lat_p50_us, lat_p99_us, lat_max_us;   /* tsorig (producer publish) -> after_frag verdict */
  unsigned long metrics[ 5 ];
  unsigned long overruns;        /* frags the GPU read after the producer had reused their line (FDGPU_VTILE_OVERRUN) */
  unsigned long tile_ns[ 4 ];    /* host time summed over tiles: frag intake (mcache polls + during_frag),
                                    after_frags, housekeep, whole tile loop */
  unsigned long verdicts;        /* frags that reached after_frag (any result) */
  unsigned long lost;            /* frags skipped by overrun tiles (unreliable link): verdicts + lost = frags */
  unsigned long batches, batch_txns, inflight_max;
  unsigned long gpu_lat_hist[ FDGPU_VTILE_LAT_BUCKETS ];   /* batch launch -> drained, summed over tiles */
  int           tiles, gpus;
  unsigned long gpu_wait_ns;     /* of tile_ns[1]: time blocked on batches not yet complete, summed over tiles */
  unsigned long poll_ns, after_ns;   /* of tile_ns[1]: non-blocking completion polls; after_frag proper */
  unsigned long launch_ns;       /* host time inside batch launches, summed over tiles (part of tile_ns[0..2]) */
  unsigned long tile_idle_ns;    /* of tile_ns[0]: intake passes that found no frag published yet */
  double        prod_seconds;    /* producers: first -> last publish */
  unsigned long prod_wait_ns;    /* producers: time waiting for credits (reliable links), summed */
  unsigned long prof_ns[ 8 ];    /* cfg.prof = 1, summed over tiles: mcache poll, during_frag, prefetch +
                                    credit, drain after_frags, housekeep after_frags, accounting, credit after
                                    after_frags, housekeep (launch decisions) */
  unsigned long copies, copy_lat_n, copy_lat_ns_sum, copy_lat_ns_max;   /* zero-copy: early GPU copies (summed over
                                    tiles; max over tiles), as fdgpu_vtile_gpu_metrics_t */
  unsigned long gather_gpu[ 8 ];  /* fdgpu_vtile_gpu_metrics_t.gather_gpu, summed (maxima: max) over tiles */
  unsigned long phase[ 9 ];       /* fdgpu_vtile_gpu_metrics_t.phase, summed (maxima: max) over tiles */
  unsigned long copy_backlog;     /* fdgpu_vtile_gpu_metrics_t.copy_backlog, summed over tiles */
  /* host contention (a shared machine): the threads' CPU time against their loops' wall time, and the
     involuntary context switches they took -- a pinned spinning thread that keeps its core shows 1.0 and 0 */
  unsigned long tile_cpu_ns, tile_wall_ns, tile_nivcsw;   /* summed over tiles */
  double        tile_cpu_share_min;                       /* the lowest tile's cpu_ns / wall_ns */
  long          tile_cpu[ 8 ];                            /* the CPUs tiles 0..7 were pinned to (-1: none) */
  unsigned long prod_cpu_ns, prod_wall_ns, prod_nivcsw;   /* summed over producers */
  unsigned long launcher[ 6 ];   /* the tiles' launch threads (cfg.launcher): commands and ns issuing them (summed),
                                    deepest queue (max), pushes that waited for room (summed), longest command (max),
                                    commands over 250 us (summed) */
  unsigned long host_copy[ 4 ];  /* the tiles' copy threads (cfg.copy_threads), fdgpu_vtile_gpu_metrics_t.host_copy summed */
  long          prod_cpu[ 4 ];   /* the CPUs producers 0..3 were pinned to (-1: none or not run) */
  unsigned long tiles_gpu_open;  /* tiles whose process had the GPU open (/dev/kfd or a /dev/dri node) when the tile
                                    finished: every tile with engine contexts of its own, no served tile */
} fdgpu_stream_stats_t;

/* The link -- mcache, in dcache (one prefilled fd_txn_m_t record per
   distinct payload), per-tile fseqs and results -- in one memory region:
   a shared file at `path` (e.g. /dev/shm/...; the creator makes it, the
   other processes fdgpu_link_join it; unlink it once fdgpu_link_joined
   reaches the process count) or, path NULL, private memory for one
   process.  The producer is a thread of whichever process passes
   run_producer to fdgpu_link_run; each process runs the tiles i % G ==
   proc on its `device`.  fdgpu_link_run returns once this process's
   tiles (and producer) are done; fdgpu_link_result then waits for every
   tile of every process and merges their results. */
typedef struct fdgpu_link fdgpu_link_t;

fdgpu_link_t *  fdgpu_link_new( char const * path, fdgpu_stream_cfg_t const * cfg, unsigned char const * payload,
                                unsigned int const * off, unsigned short const * sz, unsigned long n_payload,
                                unsigned long mcache_depth );
fdgpu_link_t *  fdgpu_link_join( char const * path, double timeout_s );
void            fdgpu_link_delete( fdgpu_link_t * link );
unsigned long   fdgpu_link_joined( fdgpu_link_t const * link );
void            fdgpu_link_cfg( fdgpu_link_t const * link, fdgpu_stream_cfg_t * cfg );
int             fdgpu_link_run( fdgpu_link_t * link, int proc, int device, int run_producer );
/* tile -> GPU binding: the tiles of process proc (i % gpus == proc), ascending, into out; returns the count */
int             fdgpu_link_tiles_of( int tiles, int gpus, int proc, int * out );
/* this process's view of the link's in mcache and in dcache (chunk c at dcache + 64 c) */
fdgpu_mcache_t * fdgpu_link_mcache( fdgpu_link_t * link );
unsigned char *  fdgpu_link_dcache( fdgpu_link_t * link );
int             fdgpu_link_result( fdgpu_link_t * link, double timeout_s, fdgpu_stream_stats_t * st );
/* Verdict trace (parity at scale, tests/test_gpu_stream_parity.py): with cap > 0 every tile this
   process runs records up to cap of its verdicts in after_frags order -- the seq and in link handed to
   during_frag, FDGPU_VTILE_* result, HA dedup tag, and for a published frag the XXH64 (seed 0)
   and size of its fd_txn_m_t record as published in the tile's out dcache.  Set before fdgpu_link_run;
   0 on success.  fdgpu_link_trace copies tile's entries out and returns their count. */
typedef struct fdgpu_link_trace {
  unsigned long seq, tag, rec_hash;
  int           result;
  unsigned int  rec_sz;
  unsigned long in_idx;
} fdgpu_link_trace_t;
int             fdgpu_link_set_trace( fdgpu_link_t * link, unsigned long cap );
unsigned long   fdgpu_link_trace( fdgpu_link_t const * link, int tile, fdgpu_link_trace_t * out, unsigned long max );
/* Always on, per tile this process runs: the first 8 verdicts that were neither published nor overrun
   (parse / verify / dedup / bundle failures; in the bench's all-valid streams each one is an anomaly),
   each with the frag's payload index in the link and the GPU batch that verified it; returns how many
   such verdicts there were. */
typedef struct fdgpu_link_anomaly {
  unsigned long seq, in_idx, payload_idx, tag;
  int           result, code;          /* FDGPU_VTILE_*, and the GPU's code (fdgpu_vtile_done_t.code) */
  unsigned int  ctx, batch_txns, batch_pos;
  int           path;                  /* FDGPU_PATH_* or latency lanes */
} fdgpu_link_anomaly_t;
unsigned long   fdgpu_link_anomalies( fdgpu_link_t const * link, int tile, fdgpu_link_anomaly_t * out, unsigned long max );
/* All of them by result: cnt[ FDGPU_VTILE_* ] (8 entries).  cnt[ FDGPU_VTILE_PUBLISH ] (never an anomaly) counts
   instead the dedup failures that are not anomalies: the link's payloads recycle, and a tile that lost or saw
   overrun most of its frags since it published a payload still holds that payload's tag at its next round (the
   reference tile's tcache drops it the same way).  Those are the dedups of a payload this tile published
   before, and they are not in the anomaly count.  Returns the anomaly count. */
unsigned long   fdgpu_link_anomaly_results( fdgpu_link_t const * link, int tile, unsigned long * cnt );

/* served tiles (cfg.svc): this process's verify service after fdgpu_link_run -- its metrics and the CPU its
   loop ran on */
int             fdgpu_link_svc_stats( fdgpu_link_t const * link, fdgpu_vsvc_stats_t * out, int * svc_cpu );
/* where the link's memory is: per producer q (returns the count) the NUMA node its in dcache part and its mcache
   got (-1 unknown), and of the link region as this process maps it the bytes in 2 MiB pages and in all */
int             fdgpu_link_placement( fdgpu_link_t const * link, int * dc_node, int * mc_node, unsigned long * huge_bytes,
                                      unsigned long * map_bytes );
/* served tiles: the tile program's body (fdgpu_tile <link> <service segment> <tile> <cpu> [copy cpus]): runs
   tile `tile` of the shared link in this process, served by the service segment at svc_path, with no GPU
   call; pinned to cpu (-1: not pinned).  0, or < 0 (the link's failure code, -10 - code). */
int             fdgpu_link_run_tile( fdgpu_link_t * link, int tile, char const * svc_path, int cpu, int const * copy_cpus,
                                     int ncopy );

/* one process, private link, every tile on `device` (G = 1) */
int             fdgpu_stream_run( int device, fdgpu_stream_cfg_t const * cfg, unsigned char const * payload,
                                  unsigned int const * off, unsigned short const * sz, unsigned long n_payload,
                                  unsigned long mcache_depth, fdgpu_stream_stats_t * st );

/* the same with a reliable link (kept for existing callers) */
int             fdgpu_stream_bench( int device, unsigned char const * payload, unsigned int const * off,
                                    unsigned short const * sz, unsigned long n_payload, unsigned long n_frags,
                                    int tiles, unsigned long batch_txn, unsigned long max_inflight,
                                    unsigned long mcache_depth, double rate_fps, int zero_copy,
                                    fdgpu_stream_stats_t * st );

#ifdef __cplusplus
}
#endif

#endif /* HEADER_fd_verify_gpu_h */
