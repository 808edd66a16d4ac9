/* fd_verify_gpu.c -- the verify tile's frag callbacks over the GPU engine,
   a minimal tango (mcache / dcache / tcache) and the streaming benchmark.
   Host C; see include/fd_verify_gpu.h for the contract and the reference
   lines each part replaces. */

#define _GNU_SOURCE
#include "../../include/fd_verify_gpu.h"
#include "../../include/fd_ed25519_gpu.h"
#include "fd_vsvc_private.h"

#include <fcntl.h>
#include <pthread.h>
#include <sched.h>
#include <x86intrin.h>
#include <stdio.h>
#include <sys/mman.h>
#include <sys/resource.h>
#include <sys/stat.h>
#include <sys/vfs.h>
#include <sys/wait.h>
#include <dirent.h>
#include <dlfcn.h>
#include <spawn.h>
#include <sys/syscall.h>
#include <unistd.h>
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

/* XXH64 of any length (the published algorithm): the link's verdict trace hashes published records */
ulong
fdgpu_xxh64( ulong seed, uchar const * p, ulong n ) {
  uchar const * e = p + n;
  ulong h;
  if( n >= 32UL ) {
    ulong v[4] = { seed + P1 + P2, seed + P2, seed, seed - P1 };
    for( ; p + 32 <= e; p += 32 ) for( int i=0; i<4; i++ ) v[i] = xxh_round( v[i], ld64( p + 8*i ) );
    h = rotl64( v[0], 1 ) + rotl64( v[1], 7 ) + rotl64( v[2], 12 ) + rotl64( v[3], 18 );
    for( int i=0; i<4; i++ ) { h ^= xxh_round( 0UL, v[i] ); h = h * P1 + P4; }
  } else h = seed + P5;
  h += n;
  for( ; p + 8 <= e; p += 8 ) { h ^= xxh_round( 0UL, ld64( p ) ); h = rotl64( h, 27 ) * P1 + P4; }
  if( p + 4 <= e ) { unsigned w; memcpy( &w, p, 4 ); h ^= (ulong)w * P1; h = rotl64( h, 23 ) * P2 + P3; p += 4; }
  for( ; p < e; p++ ) { h ^= (ulong)*p * P5; h = rotl64( h, 11 ) * P1; }
  h ^= h >> 33; h *= P2; h ^= h >> 29; h *= P3; h ^= h >> 32;
  return h;
}

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

/* start the map lines a query / insert of tag will touch, and the map line
   of the tag an insert `ahead` inserts from now would evict */
static inline void tc_prefetch( fdgpu_tcache_t const * tc, ulong tag, ulong ahead ) {
  __builtin_prefetch( &tc->map[ tc_slot( tag, tc->map_cnt ) ] );
  ulong o = tc->oldest + ahead; if( o >= tc->depth ) o %= tc->depth;
  ulong old = tc->ring[ o ];
  if( old ) __builtin_prefetch( &tc->map[ tc_slot( old, tc->map_cnt ) ], 1 );
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

/* FD_TCACHE_QUERY and, when the tag is absent and `ins`, FD_TCACHE_INSERT
   into the empty slot the query's probe ended at: one probe for both */
static inline int tc_query_insert( fdgpu_tcache_t * tc, ulong tag, int ins ) {
  if( !tag ) return 1;
  ulong i;
  if( tc_find( tc, tag, &i ) ) return 1;
  if( ins ) {
    tc->map[i] = tag;
    ulong old = tc->ring[ tc->oldest ];
    tc->ring[ tc->oldest ] = tag;
    tc->oldest = ( tc->oldest + 1UL == tc->depth ) ? 0UL : tc->oldest + 1UL;
    if( old && tc_find( tc, old, &i ) ) tc_map_remove( tc, i );
  }
  return 0;
}

int fdgpu_tcache_insert( fdgpu_tcache_t * tc, ulong tag ) { return tc_query_insert( tc, tag, 1 ); }

/* ---- mcache / dcache -------------------------------------------------
   An mcache is a ring of 32-byte frag metadata lines indexed by seq &
   (depth-1), laid out as fd_frag_meta_t (src/tango/fd_tango_base.h:
   146-203): seq, sig, chunk, sz, ctl, tsorig, tspub, the timestamps
   compressed to their low 32 bits (fd_frag_meta_ts_comp).  The producer
   marks the line in progress (seq-1), writes the fields and publishes seq
   (release); a consumer reads seq, the fields, then seq again (src/tango/
   mcache/fd_mcache.h:288-325 semantics): equal = ready, behind = not yet
   published, ahead = overrun. */

/* FDGPU_MC_PAD (A/B builds): pad each line to a 64-byte cache line, so the
   tiles that read alternate seqs never share a line */
#ifndef FDGPU_MC_PAD
#define FDGPU_MC_PAD 0
#endif
typedef struct {
  _Atomic ulong  seq;
  ulong          sig;
  unsigned       chunk;
  unsigned short sz, ctl;
  unsigned       tsorig, tspub;
#if FDGPU_MC_PAD
  unsigned char  _pad[ 32 ];
#endif
} mc_line_t;

struct fdgpu_mcache {
  ulong       depth;
  mc_line_t * line;
  int         own;          /* line[] allocated here (else it lives in a shared link or the caller's mcache) */
  int         reg;          /* registered with the GPU here (fdgpu_vtile_set_in_links), from reg_base */
  void *      reg_base;
};

/* bytes of an mcache's lines, whole pages (page-aligned line arrays can be
   registered with the GPU without sharing a page with anything else) */
static ulong mc_bytes( ulong depth ) { return ( depth * sizeof(mc_line_t) + 4095UL ) & ~4095UL; }

static void mc_init_lines( mc_line_t * line, ulong depth, ulong seq0 ) {
  memset( (void *)line, 0, depth * sizeof(mc_line_t) );
  /* every line starts "one lap behind" so seq0.. read as not yet published */
  for( ulong i=0; i<depth; i++ ) atomic_store_explicit( &line[ (seq0 + i) & (depth - 1UL) ].seq, seq0 + i - depth, memory_order_relaxed );
}

fdgpu_mcache_t *
fdgpu_mcache_new( ulong depth, ulong seq0 ) {
  if( !depth || (depth & (depth - 1UL)) ) return NULL;
  fdgpu_mcache_t * mc = (fdgpu_mcache_t *)calloc( 1, sizeof(fdgpu_mcache_t) );
  if( !mc ) return NULL;
  mc->depth = depth; mc->own = 1;
  mc->line = (mc_line_t *)aligned_alloc( 4096, mc_bytes( depth ) );
  if( !mc->line ) { free( mc ); return NULL; }
  mc_init_lines( mc->line, depth, seq0 );
  return mc;
}

/* an existing fd_frag_meta_t ring (fd_mcache_join's return, src/tango/mcache/fd_mcache.h:113,137; line
   layout src/tango/fd_tango_base.h:146-203, the same 32 bytes as mc_line_t): no copy, nothing written.
   Line of seq = seq & (depth-1), FD_MCACHE_LG_INTERLEAVE 0 (fd_mcache.h:265-272) */
fdgpu_mcache_t *
fdgpu_mcache_wrap( void * lines, ulong depth ) {
  if( !lines || !depth || (depth & (depth - 1UL)) || ( (ulong)lines & 31UL ) ) return NULL;
  fdgpu_mcache_t * mc = (fdgpu_mcache_t *)calloc( 1, sizeof(fdgpu_mcache_t) );
  if( !mc ) return NULL;
  mc->depth = depth; mc->line = (mc_line_t *)lines; mc->own = 0;
  return mc;
}

ulong fdgpu_mcache_depth( fdgpu_mcache_t const * mc ) { return mc->depth; }
void * fdgpu_mcache_lines( fdgpu_mcache_t * mc ) { return (void *)mc->line; }

void fdgpu_mcache_delete( fdgpu_mcache_t * mc ) {
  if( !mc ) return;
  if( mc->reg ) fdgpu_host_unregister( mc->reg_base );
  if( mc->own ) free( mc->line );
  free( mc );
}

static inline void
mc_publish( mc_line_t * l, ulong seq, ulong sig, unsigned chunk, unsigned sz, unsigned tsorig, unsigned tspub ) {
  atomic_store_explicit( &l->seq, seq - 1UL, memory_order_relaxed );   /* mark in-progress */
  atomic_thread_fence( memory_order_release );
  l->sig = sig; l->chunk = chunk; l->sz = (unsigned short)sz; l->ctl = 0; l->tsorig = tsorig; l->tspub = tspub;
  atomic_store_explicit( &l->seq, seq, memory_order_release );
}

void
fdgpu_mcache_publish( fdgpu_mcache_t * mc, ulong seq, ulong sig, unsigned chunk, unsigned sz, ulong tsorig, ulong tspub ) {
  mc_publish( &mc->line[ seq & (mc->depth - 1UL) ], seq, sig, chunk, sz, (unsigned)tsorig, (unsigned)tspub );
}

/* 0 ready (copied to *out), 1 not yet published, -1 overrun; *found = the
   seq the line held (where an overrun consumer resumes, fd_stem.c:590-596) */
static inline int
mc_poll( mc_line_t const * l, ulong seq, fdgpu_frag_meta_t * out, ulong * found ) {
  ulong s0 = atomic_load_explicit( (_Atomic ulong *)&l->seq, memory_order_acquire );
  *found = s0;
  if( (long)(s0 - seq) < 0 ) return 1;
  if( s0 != seq ) return -1;
  out->seq = seq; out->sig = l->sig; out->chunk = l->chunk; out->sz = l->sz; out->tsorig = l->tsorig; out->tspub = l->tspub;
  atomic_thread_fence( memory_order_acquire );
  ulong s1 = atomic_load_explicit( (_Atomic ulong *)&l->seq, memory_order_relaxed );
  *found = s1;
  return s1 == seq ? 0 : -1;                 /* overrun while reading */
}

int
fdgpu_mcache_poll( fdgpu_mcache_t const * mc, ulong seq, fdgpu_frag_meta_t * out ) {
  ulong found;
  return mc_poll( &mc->line[ seq & (mc->depth - 1UL) ], seq, out, &found );
}

int
fdgpu_mcache_query( fdgpu_mcache_t const * mc, ulong seq, fdgpu_frag_meta_t * out, ulong * seq_found ) {
  ulong found;
  int r = mc_poll( &mc->line[ seq & (mc->depth - 1UL) ], seq, out, &found );
  if( seq_found ) *seq_found = found;
  return r;
}

/* fd_frag_meta_ts_decomp: the full timestamp nearest to now whose low 32
   bits are ts (ts may lie up to 2^31 ns before or after now) */
static inline ulong ts_decomp( unsigned ts, ulong now ) { return now + (ulong)(long)(int)( ts - (unsigned)now ); }

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
  ulong seq, tsorig, chunk;              /* seq: the frag's full 64-bit seq on its in link */
  ulong bundle_id;                       /* from the frag header, read in during_frag */
  ulong cidx;                            /* zero-copy: the frag's index among context k's gathered submissions */
  unsigned short payload_sz;
  int   k;                               /* engine context the frag's batch went to */
  int   ovr;                             /* the caller's seq re-check failed after during_frag's host copy */
  int   in_idx;                          /* the in link it came from (the stem's in_idx) */
  ulong cp;                              /* host copy threads: 1 + the frag's copy task (0: none) */
} vt_pend_t;

/* Host copy threads (fdgpu_vtile_opts_t.copy_threads).  With zero-copy intake the GPU copy reads each
   record over PCIe for the verify kernels and, by default, writes it back into the out dcache: every
   record crosses the link twice, and the device-to-host direction (the write-back's 64-B writes plus
   the reads' requests) is what bounds the max-rate stream.  With copy threads the
   GPU only reads (FDGPU_GATHER_NO_WRITEBACK) and the tile's own threads copy the record in -> out
   dcache, as the reference's during_frag does with fd_memcpy (fd_verify_tile.c:96-101) -- off the
   tile's loop.  Each copy is the stem's "copy, then re-check the line" (fd_stem.c:667-686): a thread
   copies bytes [0, 10) and [12, sz) of the record (the GPU writes txn_t_sz, bytes 10-11, and the
   fd_txn_t image behind the payload), then re-reads the frag's mcache line; a changed seq marks the
   frag overrun (never published, as a frag the GPU found overrun).  Tasks go round robin to the
   threads, each an SPSC ring with a completion counter; after_frag waits for the frag's copy (it has
   long finished: the copy takes ~100 ns, the GPU batch ~1 ms) and a reliable link's credit stops at
   the first frag whose copy (GPU or host) is not known complete. */
typedef struct {
  uchar const *  src;
  uchar *        dst;
  ulong          sz;
  ulong const *  line_seq;               /* the frag's in-mcache line seq word (NULL: no check) */
  ulong          seq;
  int *          ovr;                    /* the frag's pending entry: set to 1 if the line changed */
} vt_cp_task_t;

typedef struct {
  vt_cp_task_t *   ring;
  ulong            mask;
  _Atomic ulong    tail __attribute__(( aligned( 64 ) ));   /* tasks published to the copy thread (the tile) */
  _Atomic ulong    done __attribute__(( aligned( 64 ) ));   /* tasks completed (the copy thread) */
  ulong            ptail __attribute__(( aligned( 64 ) ));  /* the tile's: tasks written (published in groups) */
  ulong            sdone;                                     /* the tile's: done as last seen */
  _Atomic int      stop;
  ulong            busy_ns, ovr_cnt;     /* the copy thread's */
  int              cpu;
  pthread_t        th;
} vt_cp_t;

/* Engine contexts per tile (fdgpu_vtile_opts_t.nctx, 1..VT_NCTX_MAX, default 2).
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
  fdgpu_launcher_t *    launcher;        /* opt.launcher: the launch thread of every context (NULL: none) */
  vt_cp_t *             cp[ FDGPU_VTILE_COPY_THREADS_MAX ];   /* opt.copy_threads: the host copy threads */
  int                   ncp;
  int                   ncp_want;        /* opt.copy_threads: started when zero-copy intake turns on (set_in_links) */
  ulong                 cp_cnt, cp_wait_ns;                   /* copy tasks pushed; time after_frags waited on one */
  int                   device, semantics;   /* to recreate a faulted context */
  int                   fault_seen[ VT_NCTX_MAX ];
  fdgpu_vtile_opts_t    opt;             /* with the defaults filled in */
  int                   gpu_tag;         /* HA dedup tags from the GPU (!opt.host_dedup_tag) */
  ulong                 min_batch, max_wait_ns, fill_t0;   /* see fdgpu_vtile_housekeep */
  /* zero-copy intake: the GPU copies of the frags (fdgpu_ed25519_gather) */
  ulong                 sub_cnt[ VT_NCTX_MAX ];            /* gathered submissions per context, cumulative */
  ulong                 copy_cursor;     /* pending-ring counter: frags below it are known to be copied */
  ulong                 copy_t0;         /* host time the oldest frag not yet given to a gather was taken (0: none) */
  ulong                 uncopied[ FDGPU_VTILE_IN_MAX ];    /* per in link: frags taken and not yet known copied */
  ulong                 uncopied_tot;                      /* ... over all links (bounded by opt.max_uncopied) */
  ulong                 copied_next[ FDGPU_VTILE_IN_MAX ]; /* per in link: 1 + seq of the last frag known copied */
  struct { ulong target, t; } cq[ VT_NCTX_MAX ][ 8 ];     /* early copies in flight: gathered count they complete at */
  ulong                 cq_head[ VT_NCTX_MAX ], cq_tail[ VT_NCTX_MAX ];
  fdgpu_vtile_gpu_metrics_t gm;
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
  ulong                 rr_idx, rr_cnt;  /* before_frag's round robin (fdgpu_vtile_set_round_robin) */
  ulong                 metrics[5];
  /* zero-copy intake (fdgpu_vtile_set_in_link): frags stay in the in
     dcache, the GPU gathers them; in_mc (optional) for the overrun check */
  int                   zc;
  fdgpu_mcache_t const * in_mcs[ FDGPU_VTILE_IN_MAX ];
  uchar const *         in_mc_dev[ FDGPU_VTILE_IN_MAX ];   /* device view of each in link's mcache lines (or NULL) */
  uchar const *         src_lo, * src_hi, * src_dev;       /* the registered region the last frag came from */
  int                   n_in;
  /* the tile's in links as the stem numbers them (fdgpu_vtile_set_in): kind and data region */
  int                   in_kind[ FDGPU_VTILE_IN_MAX ];
  uchar const *         in_mem[ FDGPU_VTILE_IN_MAX ];
  ulong                 in_chunk0[ FDGPU_VTILE_IN_MAX ], in_wmark[ FDGPU_VTILE_IN_MAX ];
  ulong                 overruns;
  /* served by a verify service (fdgpu_vtile_new_svc): no engine contexts (nctx 0); requests and completions
     through the service's rings */
  fdgpu_vsvc_t *        svc;
  vsvc_client_t *       sc;
  vsvc_req_t *          sreq;
  vsvc_cpl_t const *    scpl;
  ulong                 smask, req_pub, cpl_seen;
  int                   client, svc_dead;
  int                   gpu_rec;         /* the GPU writes each record's txn_t_sz and fd_txn_t image (zero-copy or served) */
  uchar const *         rgn_lo[ FDGPU_VSVC_RGN_MAX ];      /* the service's regions in this process */
  ulong                 rgn_sz[ FDGPU_VSVC_RGN_MAX ];
  int                   rgn_last;
  ulong                 in_line_ref[ FDGPU_VTILE_IN_MAX ]; /* each in link's mcache lines: region << 56 | offset (~0: none) */
  /* poll scratch */
  ulong                 batch;
  ulong *               p_tags;
  ulong *               p_dtag;          /* GPU-computed HA dedup tags */
  signed char *         p_codes;
  uchar *               p_img;
  unsigned short *      p_fp;
};

/* one record, bytes [0, 10) and [12, sz) of src -> dst: around txn_t_sz, which the GPU writes, and not
   past sz (the GPU writes the fd_txn_t image right behind the payload), so the two never write the same
   byte whatever their order.  (Streaming stores measured slower here: 165-180 vs 125-150 ns per record,
   profiles/r05/hc2.) */
static inline void vt_cp_record( uchar * dst, uchar const * src, ulong sz ) {
  memcpy( dst, src, 10UL );
  memcpy( dst + 12UL, src + 12UL, sz - 12UL );
}

static void * vt_cp_main( void * arg ) {
  vt_cp_t * c = (vt_cp_t *)arg;
  if( c->cpu >= 0 ) {
    cpu_set_t set; CPU_ZERO( &set ); CPU_SET( c->cpu, &set );
    (void)pthread_setaffinity_np( pthread_self(), sizeof(set), &set );
  }
  ulong j = atomic_load_explicit( &c->done, memory_order_relaxed );
  for(;;) {
    ulong t = atomic_load_explicit( &c->tail, memory_order_acquire );
    if( j == t ) {
      if( atomic_load_explicit( &c->stop, memory_order_acquire ) ) break;
      _mm_pause();
      continue;
    }
    ulong t0 = now_ns();
    for( ; j < t; j++ ) {
      vt_cp_task_t const * k = &c->ring[ j & c->mask ];
      if( j + 1UL < t ) {                                      /* the next record, whole (~21 lines, cold) */
        vt_cp_task_t const * nk = &c->ring[ ( j + 1UL ) & c->mask ];
        for( ulong o=0UL; o<nk->sz; o+=64UL ) __builtin_prefetch( nk->src + o );
      }
      vt_cp_record( k->dst, k->src, k->sz );
      if( k->line_seq ) {                                        /* the stem's re-check after its copy */
        atomic_thread_fence( memory_order_acquire );
        if( atomic_load_explicit( (_Atomic ulong const *)k->line_seq, memory_order_relaxed ) != k->seq ) {
          *k->ovr = 1; c->ovr_cnt++;
        }
      }
    }
    atomic_store_explicit( &c->done, j, memory_order_release );
    c->busy_ns += now_ns() - t0;
  }
  return NULL;
}

static void vt_cp_delete( vt_cp_t * c ) {
  if( !c ) return;
  atomic_store_explicit( &c->stop, 1, memory_order_release );
  pthread_join( c->th, NULL );
  free( c->ring ); free( c );
}

static vt_cp_t * vt_cp_new( ulong cap, int cpu ) {
  vt_cp_t * c = (vt_cp_t *)calloc( 1, sizeof(vt_cp_t) );
  if( !c ) return NULL;
  c->mask = pow2_up( cap ) - 1UL; c->cpu = cpu;
  c->ring = (vt_cp_task_t *)calloc( c->mask + 1UL, sizeof(vt_cp_task_t) );
  if( !c->ring || pthread_create( &c->th, NULL, vt_cp_main, c ) ) { free( c->ring ); free( c ); return NULL; }
  return c;
}

/* copy task k (1-based, vt_pend_t.cp) has completed.  The tile keeps the last completion count it saw and
   reads the thread's (a line the thread keeps writing) only when that is not enough: one cross-core read
   per batch of verdicts instead of one per frag */
static inline int vt_cp_done( fdgpu_vtile_t const * vt, ulong k ) {
  ulong i = k - 1UL;
  vt_cp_t * c = vt->cp[ i % (ulong)vt->ncp ];
  ulong j = i / (ulong)vt->ncp;
  if( c->sdone > j ) return 1;
  if( c->ptail > atomic_load_explicit( &c->tail, memory_order_relaxed ) )   /* unpublished tasks: publish them */
    atomic_store_explicit( &c->tail, c->ptail, memory_order_release );
  c->sdone = atomic_load_explicit( &c->done, memory_order_acquire );
  return c->sdone > j;
}

/* publish the tasks written so far to every copy thread (the tile publishes them in groups of 16) */
static inline void vt_cp_publish( fdgpu_vtile_t const * vt ) {
  for( int i=0; i<vt->ncp; i++ ) {
    vt_cp_t * c = vt->cp[i];
    if( c->ptail != atomic_load_explicit( &c->tail, memory_order_relaxed ) )
      atomic_store_explicit( &c->tail, c->ptail, memory_order_release );
  }
}

/* wait for frag p's host copy, if it has one (copy threads; in practice long done) */
static inline void vt_cp_wait( fdgpu_vtile_t * vt, vt_pend_t const * p ) {
  if( !p->cp || vt_cp_done( vt, p->cp ) ) return;
  ulong tw = now_ns();
  while( !vt_cp_done( vt, p->cp ) ) _mm_pause();
  vt->cp_wait_ns += now_ns() - tw;
}

/* ---- a tile served by a verify service (fdgpu_vtile_new_svc) ----------------------------------------
   during_frag writes one request per frag (index = the frag's pending index) and publishes the ring's
   tail in groups of 16 and at every housekeep / flush / drain; after_frags reads the completions, which
   come back in request order. */

static inline void vt_svc_publish( fdgpu_vtile_t * vt ) {
  if( vt->req_pub != vt->pend_tail ) {
    vt->req_pub = vt->pend_tail;
    atomic_store_explicit( &vt->sc->req_tail, vt->req_pub, memory_order_release );
  }
}

/* 1 if the service failed to start or stopped beating: nothing more will complete */
static int vt_svc_dead( fdgpu_vtile_t * vt ) {
  if( vt->svc_dead ) return 1;
  vsvc_hdr_t * h = vt->svc->h;
  int r = atomic_load_explicit( &h->ready, memory_order_acquire );
  if( r < 0 ) { vt->svc_dead = 1; return 1; }
  if( r == 0 ) return 0;                               /* not started yet: requests wait */
  ulong hb = atomic_load_explicit( &h->heartbeat, memory_order_acquire ), now = now_ns();
  if( now > hb && now - hb > VSVC_DEAD_NS ) { vt->svc_dead = 1; return 1; }
  return 0;
}

/* the request of the frag about to be taken (pending index pend_tail) */
static inline void vt_svc_req( fdgpu_vtile_t * vt, ulong src, ulong line, ulong seq, ulong rec_sz, unsigned flags ) {
  vsvc_req_t * r = &vt->sreq[ vt->pend_tail & vt->smask ];
  r->seq = seq; r->src = src; r->line = line; r->dst_chunk = (unsigned)vt->out_chunk;
  r->rec_sz = (unsigned short)rec_sz; r->flags = (unsigned short)flags;
}

/* region id << 56 | offset of [p, p+n) among the service's regions as this process maps them, ~0UL if outside */
static ulong vt_svc_ref( fdgpu_vtile_t * vt, void const * p, ulong n ) {
  uchar const * q = (uchar const *)p;
  int i = vt->rgn_last;
  if( vt->rgn_lo[i] && q >= vt->rgn_lo[i] && q + n <= vt->rgn_lo[i] + vt->rgn_sz[i] )
    return ( (ulong)i << 56 ) | (ulong)( q - vt->rgn_lo[i] );
  for( i=0; i<FDGPU_VSVC_RGN_MAX; i++ )
    if( vt->rgn_lo[i] && q >= vt->rgn_lo[i] && q + n <= vt->rgn_lo[i] + vt->rgn_sz[i] ) {
      vt->rgn_last = i;
      return ( (ulong)i << 56 ) | (ulong)( q - vt->rgn_lo[i] );
    }
  return ~0UL;
}

/* one engine context of the tile.  Adaptive batching launches a partial
   batch when the GPU has room (low load: the latency path) and a full one
   when frags back up (high load: the throughput path, whose per-signature
   work is 0.5x the 4-lane DSM's). */
static fdgpu_ed25519_ctx_t *
vt_ctx_new( fdgpu_vtile_t const * vt, int k ) {
  ulong b = vt->batch;
  fdgpu_ed25519_ctx_t * c = fdgpu_ed25519_ctx_new( vt->device, b, 16UL*b, b*2304UL + 1024UL, vt->semantics );
  if( c ) {
    /* latency path for batches up to half the batch limit (opt.small_max overrides) */
    ulong sm = fdgpu_ed25519_set_small_batch_max( c, 0UL );
    fdgpu_ed25519_set_small_batch_max( c, vt->opt.small_max ? vt->opt.small_max : ( sm < b/2UL ? sm : b/2UL ) );
    /* the GPU computes the HA dedup tags and, for gathered records, stores
       txn_t_sz: after_frag then touches neither payload nor record */
    fdgpu_ed25519_set_dedup( c, vt->gpu_tag, vt->seed );
    unsigned parts = vt->opt.cu_split ? (unsigned)vt->nctx : 1u, part = vt->opt.cu_split ? (unsigned)k : 0u;
    if( vt->opt.gather_cus && fdgpu_ed25519_reserve_cus( c, vt->opt.gather_cus, part, parts ) ) {
      fdgpu_ed25519_ctx_delete( c ); return NULL;
    }
    /* 0 = default: on -- unless the engine's test hook (fdgpu_debug_opts_t.cu_exclusive) already chose a
       mode for new contexts, which the tile then keeps (the tile tests' latency8 / latency8x paths) */
    int excl = vt->opt.cu_exclusive ? vt->opt.cu_exclusive : ( fdgpu_ed25519_get_cu_exclusive( c ) ? 0 : 1 );
    if( excl > 0 && fdgpu_ed25519_set_cu_exclusive( c, excl ) ) { fdgpu_ed25519_ctx_delete( c ); return NULL; }
    /* each context's exclusive walk within its share of the CUs (the contexts' batches overlap; with cu_split
       the share is the context's own part): a walk wider than its share would wait on the other context's
       workgroups and hold the gathers queued behind it (profiles/r05/cb) */
    unsigned share = vt->opt.lat_share > 0 ? (unsigned)vt->opt.lat_share : vt->opt.lat_share < 0 ? 0u : (unsigned)vt->nctx;
    /* by the context's actual mode: also when the engine's test hook chose it (excl 0 here) -- any mode with an
       exclusive walk (1..3) gets its share */
    int mode = fdgpu_ed25519_get_cu_exclusive( c );
    if( mode >= 1 && mode <= 3 && fdgpu_ed25519_set_lat_share( c, share ) ) {
      fdgpu_ed25519_ctx_delete( c ); return NULL;
    }
    fdgpu_ed25519_set_record_fp_off( c, 10 );          /* offsetof( fd_txn_m_t, txn_t_sz ) */
    /* every staging buffer and the gather stream now: batches then allocate nothing (the tile's sandbox
       allows no allocation it does not need, fd_verify_gpu_tile.seccomppolicy) */
    if( fdgpu_ed25519_prepare( c, 1 ) ) { fdgpu_ed25519_ctx_delete( c ); return NULL; }
    if( vt->launcher && fdgpu_ed25519_set_launcher( c, vt->launcher ) ) { fdgpu_ed25519_ctx_delete( c ); return NULL; }
  }
  return c;
}

fdgpu_vtile_t *
fdgpu_vtile_new( int device, ulong batch_txn, ulong tcache_depth, ulong seed, ulong out_dcache_bytes, int semantics ) {
  return fdgpu_vtile_new_opts( device, batch_txn, tcache_depth, seed, out_dcache_bytes, semantics, NULL );
}

fdgpu_vtile_t *
fdgpu_vtile_new_opts( int device, ulong batch_txn, ulong tcache_depth, ulong seed, ulong out_dcache_bytes, int semantics,
                      fdgpu_vtile_opts_t const * opts ) {
  if( !batch_txn || !tcache_depth || out_dcache_bytes < 8UL*VT_RESERVE_MAX ) return NULL;
  fdgpu_vtile_t * vt = (fdgpu_vtile_t *)calloc( 1, sizeof(fdgpu_vtile_t) );
  if( !vt ) return NULL;
  if( opts ) vt->opt = *opts;
  if( !vt->opt.nctx )         vt->opt.nctx = 2;
  if( !vt->opt.max_wait_ns )  vt->opt.max_wait_ns = 2000000UL;
  if( !vt->opt.copy_wait_ns ) vt->opt.copy_wait_ns = FDGPU_VTILE_COPY_WAIT_NS;
  if( !vt->opt.copy_min )     vt->opt.copy_min = FDGPU_VTILE_COPY_MIN;
  if( !vt->opt.max_uncopied ) vt->opt.max_uncopied = FDGPU_VTILE_MAX_UNCOPIED;
  /* staging arena of a batch = its range of the out dcache (in-place submits): up to
     batch_txn records of at most VT_RESERVE_MAX bytes (rounded to chunk pairs) */
  vt->nctx = vt->opt.nctx;
  if( vt->nctx < 1 ) vt->nctx = 1;
  if( vt->nctx > VT_NCTX_MAX ) vt->nctx = VT_NCTX_MAX;
  vt->opt.nctx = vt->nctx;
  vt->batch_ns = 500e3;
  vt->device = device; vt->semantics = semantics; vt->batch = batch_txn; vt->seed = seed;
  vt->gpu_tag = !vt->opt.host_dedup_tag;
  vt->min_batch = vt->opt.min_batch; vt->max_wait_ns = vt->opt.max_wait_ns;
  if( vt->opt.launcher && !( vt->launcher = fdgpu_launcher_new( device, vt->opt.launcher_core - 1 ) ) ) {
    free( vt ); return NULL;
  }
  int ctx_ok = 1;
  for( int k=0; k<vt->nctx; k++ ) if( !( vt->ctx[k] = vt_ctx_new( vt, k ) ) ) ctx_ok = 0;
  vt->tcache = fdgpu_tcache_new( tcache_depth );
  ulong nchunk = ( out_dcache_bytes / FDGPU_CHUNK_SZ ) & ~1UL;
  vt->dcache = (uchar *)fdgpu_host_alloc( nchunk * FDGPU_CHUNK_SZ );   /* pinned: batches upload from it in place */
  ulong rchunk = ( ( VT_RESERVE_MAX + 127UL ) >> 7 ) << 1;
  vt->chunk0 = 0UL; vt->wmark = nchunk - rchunk; vt->out_chunk = 0UL;
  /* frags in flight: the ring must hold them all plus one wrap's waste */
  vt->pend_cap = nchunk / rchunk - 2UL;
  vt->pend = (vt_pend_t *)calloc( vt->pend_cap, sizeof(vt_pend_t) );
  vt->seed = seed;
  vt->p_tags = (ulong *)malloc( batch_txn * sizeof(ulong) );
  vt->p_dtag = (ulong *)malloc( batch_txn * sizeof(ulong) );
  vt->p_codes = (signed char *)malloc( batch_txn );
  vt->p_img = (uchar *)malloc( batch_txn * FDGPU_TXN_IMG_STRIDE );
  vt->p_fp = (unsigned short *)malloc( batch_txn * sizeof(unsigned short) );
  int cp_ok = 1;
  if( vt->opt.copy_threads > FDGPU_VTILE_COPY_THREADS_MAX ) vt->opt.copy_threads = FDGPU_VTILE_COPY_THREADS_MAX;
  if( vt->opt.copy_threads < 0 ) vt->opt.copy_threads = 0;
  /* the copy threads only serve zero-copy intake: they start with it (fdgpu_vtile_set_in_links), so a tile
     without it has none spinning */
  vt->ncp_want = vt->opt.copy_threads;
  vt->gpu_rec = 0;
  if( !ctx_ok || !cp_ok || !vt->tcache || !vt->dcache || !vt->pend || !vt->p_tags || !vt->p_dtag || !vt->p_codes || !vt->p_img || !vt->p_fp ) {
    fdgpu_vtile_delete( vt );
    return NULL;
  }
  return vt;
}

fdgpu_vtile_t *
fdgpu_vtile_new_svc( fdgpu_vsvc_t * svc, int client, ulong tcache_depth, ulong seed, fdgpu_vtile_opts_t const * opts ) {
  if( !svc || client < 0 || client >= svc->h->clients || !tcache_depth ) return NULL;
  vsvc_client_t * k = &svc->h->client[ client ];
  int want = 0;
  if( !atomic_compare_exchange_strong( &k->state, &want, 3 ) ) return NULL;     /* 3: being attached */
  fdgpu_vtile_t * vt = (fdgpu_vtile_t *)calloc( 1, sizeof(fdgpu_vtile_t) );
  if( !vt ) { atomic_store( &k->state, 0 ); return NULL; }
  if( opts ) vt->opt = *opts;
  if( !vt->opt.copy_wait_ns ) vt->opt.copy_wait_ns = FDGPU_VTILE_COPY_WAIT_NS;
  if( !vt->opt.copy_min )     vt->opt.copy_min = FDGPU_VTILE_COPY_MIN;
  if( !vt->opt.max_uncopied ) vt->opt.max_uncopied = FDGPU_VTILE_MAX_UNCOPIED;
  vt->svc = svc; vt->sc = k; vt->client = client; vt->nctx = 0; vt->opt.nctx = 0;
  vt->sreq = (vsvc_req_t *)( svc->base + k->off_req ); vt->scpl = (vsvc_cpl_t const *)( svc->base + k->off_cpl );
  vt->smask = k->ring_cap - 1UL;
  vt->req_pub = vt->cpl_seen = 0UL;
  vt->gpu_tag = !vt->opt.host_dedup_tag; vt->gpu_rec = 1;
  vt->seed = seed; vt->batch = 0UL; vt->device = -1;
  for( int i=0; i<FDGPU_VTILE_IN_MAX; i++ ) vt->in_line_ref[i] = ~0UL;
  vt->tcache = fdgpu_tcache_new( tcache_depth );
  vt->dcache = svc->base + k->off_out;
  ulong nchunk = ( k->out_sz / FDGPU_CHUNK_SZ ) & ~1UL;
  ulong rchunk = ( ( VT_RESERVE_MAX + 127UL ) >> 7 ) << 1;
  vt->chunk0 = 0UL; vt->wmark = nchunk - rchunk; vt->out_chunk = 0UL;
  vt->pend_cap = nchunk / rchunk - 2UL;                 /* (the service sized the rings for exactly this) */
  vt->pend = (vt_pend_t *)calloc( vt->pend_cap, sizeof(vt_pend_t) );
  int cp_ok = 1;
  if( vt->opt.copy_threads > FDGPU_VTILE_COPY_THREADS_MAX ) vt->opt.copy_threads = FDGPU_VTILE_COPY_THREADS_MAX;
  if( vt->opt.copy_threads < 0 ) vt->opt.copy_threads = 0;
  if( !vt->tcache || !vt->pend || vt->pend_cap + 2UL > k->ring_cap ) cp_ok = 0;
  if( cp_ok ) vt->ncp_want = vt->opt.copy_threads;      /* started with zero-copy intake (fdgpu_vtile_set_in_links) */
  if( !cp_ok ) {
    fdgpu_tcache_delete( vt->tcache ); free( vt->pend ); free( vt );
    atomic_store( &k->state, 0 );
    return NULL;
  }
  k->seed = seed; k->pid = (long)getpid();
  atomic_store_explicit( &k->state, 1, memory_order_release );
  return vt;
}

int
fdgpu_vtile_set_svc_region( fdgpu_vtile_t * vt, int id, void const * base, ulong sz ) {
  if( !vt->svc || id < 0 || id >= FDGPU_VSVC_RGN_MAX || !base ) return -1;
  if( vt->pend_tail != vt->pend_head ) return -1;      /* only while idle */
  ulong have = vt->svc->h->rgn_sz[ id ];
  if( have && sz > have ) return -1;                     /* larger than the service's region */
  vt->rgn_lo[ id ] = (uchar const *)base; vt->rgn_sz[ id ] = sz;
  return 0;
}

void
fdgpu_vtile_delete( fdgpu_vtile_t * vt ) {
  if( !vt ) return;
  if( vt->svc ) {                                        /* served: no contexts, the out dcache is the segment's */
    vt_svc_publish( vt );
    for( int i=0; i<vt->ncp; i++ ) vt_cp_delete( vt->cp[i] );
    fdgpu_tcache_delete( vt->tcache );
    free( vt->pend );
    atomic_store_explicit( &vt->sc->state, 2, memory_order_release );
    free( vt );
    return;
  }
  for( int k=0; k<VT_NCTX_MAX; k++ ) if( vt->ctx[k] ) fdgpu_ed25519_ctx_delete( vt->ctx[k] );
  fdgpu_launcher_delete( vt->launcher );       /* after its contexts: each drained its commands first */
  for( int i=0; i<vt->ncp; i++ ) vt_cp_delete( vt->cp[i] );   /* (a thread finishes its queued copies first) */
  fdgpu_tcache_delete( vt->tcache );
  fdgpu_host_free( vt->dcache ); free( vt->pend ); free( vt->p_tags ); free( vt->p_dtag ); free( vt->p_codes ); free( vt->p_img );
  free( vt->p_fp );
  free( vt );
}

uchar * fdgpu_vtile_out_dcache( fdgpu_vtile_t * vt ) { return vt->dcache; }
ulong   fdgpu_vtile_pending( fdgpu_vtile_t const * vt ) { return vt->pend_tail - vt->pend_head; }
void    fdgpu_vtile_metrics( fdgpu_vtile_t const * vt, ulong out[ 5 ] ) { memcpy( out, vt->metrics, sizeof(vt->metrics) ); }
/* bookkeeping of a batch launch on context k (filling txns) */
static void
vt_launched( fdgpu_vtile_t * vt, int k, ulong now, ulong filling ) {
  (void)filling;
  vt->launch_ns[k] = now; vt->busy[k] = 1;
  ulong f, infl = 0UL;
  for( int j=0; j<vt->nctx; j++ ) { ulong i; fdgpu_ed25519_pipeline_state( vt->ctx[j], &f, &i ); infl += i; }
  if( infl > vt->gm.inflight_max ) vt->gm.inflight_max = infl;
}

int
fdgpu_vtile_flush( fdgpu_vtile_t * vt ) {
  vt_fence();
  if( vt->svc ) {                                   /* the service launches its filling batches */
    vt_svc_publish( vt );
    atomic_fetch_add_explicit( &vt->sc->flush, 1UL, memory_order_release );
    return vt_svc_dead( vt ) ? -1 : 0;
  }
  int rc = 0;
  for( int i=0; i<vt->nctx; i++ ) {            /* oldest first: the fill context's batch is the newest */
    int k = ( vt->fill + 1 + i ) % vt->nctx;
    ulong filling, inflight;
    if( fdgpu_ed25519_faulted( vt->ctx[k] ) ) continue;
    fdgpu_ed25519_pipeline_state( vt->ctx[k], &filling, &inflight );
    if( !filling ) continue;
    if( fdgpu_ed25519_flush( vt->ctx[k] ) ) rc = -1;
    else vt_launched( vt, k, now_ns(), filling );
  }
  return rc;
}

void
fdgpu_vtile_pipeline_state( fdgpu_vtile_t const * vt, ulong * filling, ulong * inflight ) {
  *filling = 0UL; *inflight = 0UL;
  if( vt->svc ) {                                   /* served: not yet taken by the service / taken, no verdict yet */
    ulong tk = atomic_load_explicit( &vt->sc->taken, memory_order_relaxed );
    ulong cp = atomic_load_explicit( &vt->sc->cpl_tail, memory_order_relaxed );
    *filling = vt->pend_tail > tk ? vt->pend_tail - tk : 0UL; *inflight = tk > cp ? tk - cp : 0UL;
    return;
  }
  for( int k=0; k<vt->nctx; k++ ) {
    ulong f, i;
    fdgpu_ed25519_pipeline_state( vt->ctx[k], &f, &i );
    *filling += f; *inflight += i;
  }
}
ulong   fdgpu_vtile_overruns( fdgpu_vtile_t const * vt ) { return vt->overruns; }

int
fdgpu_vtile_faulted( fdgpu_vtile_t const * vt ) {
  if( vt->svc )                                     /* the service's contexts faulted now (+1: the service is gone) */
    return atomic_load_explicit( &vt->svc->h->faulted, memory_order_relaxed ) + ( vt->svc_dead ? 1 : 0 );
  int n = 0;
  for( int k=0; k<vt->nctx; k++ ) n += fdgpu_ed25519_faulted( vt->ctx[k] ) != 0;
  return n;
}

int
fdgpu_vtile_recover( fdgpu_vtile_t * vt ) {
  if( vt->svc ) return vt->svc_dead ? -2 : 0;       /* the service recreates its faulted contexts itself */
  int rc = 0;
  for( int k=0; k<vt->nctx; k++ ) {
    if( !fdgpu_ed25519_faulted( vt->ctx[k] ) ) continue;
    int busy = 0;
    for( ulong q=vt->pend_head; q<vt->pend_tail && !busy; q++ ) busy = vt->pend[ q % vt->pend_cap ].k == k;
    if( busy ) { rc = -1; continue; }
    /* the replacement first: if it cannot be made, the faulted context stays (and stays skipped) */
    fdgpu_ed25519_ctx_t * c = vt_ctx_new( vt, k );
    if( !c ) { if( !rc ) rc = -2; continue; }
    fdgpu_ed25519_ctx_delete( vt->ctx[k] );
    vt->ctx[k] = c;
    vt->busy[k] = 0; vt->fault_seen[k] = 0; vt->sub_cnt[k] = 0UL; vt->cq_head[k] = vt->cq_tail[k] = 0UL;
  }
  return rc;
}

void
fdgpu_vtile_debug_fault( fdgpu_vtile_t * vt, int k ) {
  if( vt->svc ) { if( k >= 0 && k < VSVC_NCTX_MAX ) atomic_fetch_or_explicit( &vt->sc->dbg_fault, 1 << k, memory_order_release ); return; }
  if( k >= 0 && k < vt->nctx ) fdgpu_ed25519_debug_fault( vt->ctx[k] );
}

void
fdgpu_vtile_debug_fail_launch( fdgpu_vtile_t * vt, int k ) {
  if( !vt->svc && k >= 0 && k < vt->nctx ) fdgpu_ed25519_debug_fail_launch( vt->ctx[k], 1 );
}

void
fdgpu_vtile_gpu_metrics( fdgpu_vtile_t * vt, fdgpu_vtile_gpu_metrics_t * out ) {
  *out = vt->gm;
  ulong f, i, infl = 0UL;
  memset( out->lat_hist, 0, sizeof(out->lat_hist) );
  out->batches = out->batch_txns = out->launch_ns = 0UL;
  memset( out->gather_gpu, 0, sizeof(out->gather_gpu) );
  memset( out->phase, 0, sizeof(out->phase) );
  for( int k=0; k<vt->nctx; k++ ) {
    fdgpu_ed25519_pipeline_state( vt->ctx[k], &f, &i ); infl += i;
    /* the engine counts every launch (a full slot launches inside submit) and times each batch */
    ulong b, t, h[ FDGPU_LAT_BUCKETS ];
    fdgpu_ed25519_batch_stats( vt->ctx[k], &b, &t, h );
    ulong lns, nl; fdgpu_ed25519_launch_stats( vt->ctx[k], &lns, &nl ); out->launch_ns += lns;
    ulong gs[8]; fdgpu_ed25519_gather_stats( vt->ctx[k], gs );
    out->gather_gpu[0] += gs[0]; out->gather_gpu[1] += gs[1]; out->gather_gpu[3] += gs[3]; out->gather_gpu[5] += gs[5];
    out->gather_gpu[7] += gs[7];
    if( gs[2] > out->gather_gpu[2] ) out->gather_gpu[2] = gs[2];
    if( gs[4] > out->gather_gpu[4] ) out->gather_gpu[4] = gs[4];
    if( gs[6] > out->gather_gpu[6] ) out->gather_gpu[6] = gs[6];
    ulong ph[9]; fdgpu_ed25519_phase_stats( vt->ctx[k], ph );
    for( int j=0; j<9; j++ ) {
      if( j == 2 || j == 4 || j == 6 ) { if( ph[j] > out->phase[j] ) out->phase[j] = ph[j]; }
      else out->phase[j] += ph[j];
    }
    out->batches += b; out->batch_txns += t;
    for( int j=0; j<FDGPU_LAT_BUCKETS; j++ ) out->lat_hist[j] += h[j];
  }
  if( vt->launcher ) fdgpu_launcher_stats( vt->launcher, out->launcher );
  else memset( out->launcher, 0, sizeof(out->launcher) );
  memset( out->host_copy, 0, sizeof(out->host_copy) );
  for( int i=0; i<vt->ncp; i++ ) {
    out->host_copy[0] += atomic_load_explicit( &vt->cp[i]->done, memory_order_acquire );
    out->host_copy[1] += vt->cp[i]->busy_ns; out->host_copy[2] += vt->cp[i]->ovr_cnt;
  }
  out->host_copy[3] = vt->cp_wait_ns;
  out->inflight = infl;
  out->pending = vt->pend_tail - vt->pend_head;
  out->overruns = vt->overruns;
}

int
fdgpu_vtile_set_in_link( fdgpu_vtile_t * vt, fdgpu_mcache_t const * in_mc ) {
  return fdgpu_vtile_set_in_links( vt, &in_mc, 1 );
}

int
fdgpu_vtile_set_in_links( fdgpu_vtile_t * vt, fdgpu_mcache_t const * const * in_mc, int n ) {
  if( vt->pend_tail != vt->pend_head ) return -1;       /* switch only while idle */
  if( n < 1 || n > FDGPU_VTILE_IN_MAX ) return -1;
  /* served: the service maps the lines (no GPU call here); each in link's lines must lie in one of its
     regions (fdgpu_vtile_set_svc_region) */
  for( int i=0; i<n && vt->svc; i++ ) {
    fdgpu_mcache_t const * mc = in_mc[i];
    vt->in_line_ref[i] = mc ? vt_svc_ref( vt, mc->line, mc->depth * sizeof(mc_line_t) ) : ~0UL;
    if( mc && vt->in_line_ref[i] == ~0UL ) return -2;
  }
  /* the GPU re-reads each frag's mcache line after its copy: the lines must be mapped for it */
  for( int i=0; i<n && !vt->svc; i++ ) {
    fdgpu_mcache_t * mc = (fdgpu_mcache_t *)in_mc[i];
    if( !mc || mc->reg ) continue;
    /* the lines' whole pages (an fd_mcache's lines start 256 bytes into its region, not on a page).  Already
       mapped by a larger registration (the integrator registered the mcache's workspace as a whole, as
       INTEGRATION.md does): nothing to do.  Mapped by exactly these pages (another handle on the same ring):
       one more reference, so deleting either handle leaves the other's mapping.  Partly mapped: refused --
       registering the page range would overlap the other registration (register the workspace instead). */
    ulong lo = (ulong)mc->line & ~4095UL, hi = ( (ulong)mc->line + mc->depth * sizeof(mc_line_t) + 4095UL ) & ~4095UL;
    void * b = NULL, * d = NULL; ulong rs = 0UL;
    int have = !fdgpu_host_region( (void const *)lo, &b, &rs, &d ) && (ulong)b + rs >= hi;
    if( have && !( (ulong)b == lo && rs == hi - lo ) ) continue;             /* inside a larger registration */
    if( !have && fdgpu_host_dev_ptr( mc->line, mc->depth * sizeof(mc_line_t) ) ) continue;   /* lines covered */
    int rc = fdgpu_host_register_shared( (void *)lo, hi - lo );            /* exactly these pages: shared */
    if( rc < 0 ) return -2;
    if( rc == 0 ) { mc->reg = 1; mc->reg_base = (void *)lo; }              /* (1: an owner's registration) */
  }
  /* the copy threads (opt.copy_threads), now that zero-copy intake needs them: a thread's ring holds every
     task of the pending frags it may have (round robin: pend_cap / n + 1) */
  for( int i=vt->ncp; i<vt->ncp_want; i++ ) {
    if( !( vt->cp[i] = vt_cp_new( vt->pend_cap / (ulong)vt->ncp_want + 2UL, vt->opt.copy_cores[i] - 1 ) ) ) return -3;
    vt->ncp = i + 1;
  }
  vt->zc = 1; vt->n_in = n; vt->gpu_rec = 1;
  for( int i=0; i<FDGPU_VTILE_IN_MAX; i++ ) {
    vt->in_mcs[i] = i < n ? in_mc[i] : NULL;
    vt->in_mc_dev[i] = vt->in_mcs[i] ? (uchar const *)fdgpu_host_dev_ptr( vt->in_mcs[i]->line, 8UL ) : NULL;
  }
  vt->src_lo = vt->src_hi = vt->src_dev = NULL;
  for( int i=0; i<FDGPU_VTILE_IN_MAX; i++ ) { vt->uncopied[i] = 0UL; vt->copied_next[i] = 0UL; }
  vt->uncopied_tot = 0UL;
  vt->copy_cursor = vt->pend_tail; vt->copy_t0 = 0UL;
  return 0;
}

/* a frag's copy has completed (or it left the pipeline without one) */
static inline void vt_copied( fdgpu_vtile_t * vt, vt_pend_t const * p ) {
  int l = p->in_idx;
  vt->uncopied[l]--; vt->uncopied_tot--; vt->copied_next[l] = p->seq + 1UL;
}

/* an early copy of context k was launched (for its latency metric) */
static void vt_copy_launched( fdgpu_vtile_t * vt, int k ) {
  vt->gm.copies++;
  if( vt->cq_tail[k] - vt->cq_head[k] >= 8UL ) return;   /* (not timed) */
  vt->cq[k][ vt->cq_tail[k] % 8UL ].target = fdgpu_ed25519_gather_launched( vt->ctx[k] );
  vt->cq[k][ vt->cq_tail[k] % 8UL ].t = now_ns();
  vt->cq_tail[k]++;
}

/* advance copy_cursor over the frags whose gathers have completed */
static void vt_copy_poll( fdgpu_vtile_t * vt ) {
  if( !vt->zc ) return;
  if( vt->svc ) {                                   /* the service's copied prefix of this tile's requests */
    ulong g = atomic_load_explicit( &vt->sc->copied, memory_order_acquire );
    if( vt->copy_cursor < vt->pend_head ) vt->copy_cursor = vt->pend_head;
    while( vt->copy_cursor < vt->pend_tail && vt->copy_cursor < g ) {
      vt_pend_t const * p = &vt->pend[ vt->copy_cursor % vt->pend_cap ];
      if( p->cp && !vt_cp_done( vt, p->cp ) ) break;
      vt_copied( vt, p );
      vt->copy_cursor++;
    }
    return;
  }
  ulong g[ VT_NCTX_MAX ], now = 0UL;
  for( int k=0; k<vt->nctx; k++ ) {
    g[k] = fdgpu_ed25519_gathered( vt->ctx[k] );
    while( vt->cq_head[k] < vt->cq_tail[k] && vt->cq[k][ vt->cq_head[k] % 8UL ].target <= g[k] ) {
      if( !now ) now = now_ns();
      ulong lat = now - vt->cq[k][ vt->cq_head[k] % 8UL ].t;
      vt->gm.copy_lat_ns_sum += lat; vt->gm.copy_lat_n++;
      if( lat > vt->gm.copy_lat_ns_max ) vt->gm.copy_lat_ns_max = lat;
      vt->cq_head[k]++;
    }
  }
  if( vt->copy_cursor < vt->pend_head ) vt->copy_cursor = vt->pend_head;   /* (after_frags accounts those) */
  while( vt->copy_cursor < vt->pend_tail ) {
    vt_pend_t const * p = &vt->pend[ vt->copy_cursor % vt->pend_cap ];
    if( p->cidx >= g[ p->k ] ) break;
    if( p->cp && !vt_cp_done( vt, p->cp ) ) break;            /* its host copy (copy threads) not done yet */
    vt_copied( vt, p );
    vt->copy_cursor++;
  }
}

int
fdgpu_vtile_copy( fdgpu_vtile_t * vt, int blocking ) {
  if( !vt->zc ) return 0;
  if( vt->svc ) {
    vt_cp_publish( vt );
    vt_svc_publish( vt );
    atomic_fetch_add_explicit( &vt->sc->gather, 1UL, memory_order_release );
    vt->copy_t0 = 0UL;
    vt_copy_poll( vt );
    while( blocking && vt->copy_cursor < vt->pend_tail ) {
      if( vt_svc_dead( vt ) ) return -3;
      _mm_pause();
      vt_copy_poll( vt );
    }
    return 0;
  }
  int rc = 0;
  for( int k=0; k<vt->nctx; k++ ) {
    if( fdgpu_ed25519_faulted( vt->ctx[k] ) ) continue;
    long n = fdgpu_ed25519_gather( vt->ctx[k] );
    if( n < 0 ) { rc = (int)n; continue; }
    if( n ) vt_copy_launched( vt, k );
    if( blocking && fdgpu_ed25519_gather_wait( vt->ctx[k] ) ) rc = -3;
  }
  vt->copy_t0 = 0UL;
  vt_copy_poll( vt );
  return rc;
}

ulong
fdgpu_vtile_copy_state( fdgpu_vtile_t const * vt, int link, ulong * copied_next ) {
  if( link < 0 || link >= FDGPU_VTILE_IN_MAX ) { *copied_next = 0UL; return 0UL; }
  *copied_next = vt->copied_next[link];
  return vt->uncopied[link];
}

ulong
fdgpu_vtile_oldest_pending_seq( fdgpu_vtile_t const * vt, ulong * in_idx ) {
  if( vt->pend_head >= vt->pend_tail ) { if( in_idx ) *in_idx = ~0UL; return ~0UL; }
  vt_pend_t const * p = &vt->pend[ vt->pend_head % vt->pend_cap ];
  if( in_idx ) *in_idx = (ulong)p->in_idx;
  return p->seq;
}

/* launch decision of housekeep: 1 if context f's filling batch should go now */
static int
vt_should_launch( fdgpu_vtile_t * vt, int f, ulong max_inflight, ulong now, ulong * filling ) {
  ulong inflight;
  if( fdgpu_ed25519_faulted( vt->ctx[f] ) ) return 0;
  fdgpu_ed25519_pipeline_state( vt->ctx[f], filling, &inflight );
  /* keep at least one staging slot free to accumulate in: with every slot
     in flight, each freed slot would be relaunched after a handful of
     frags and the pipeline would degenerate into tiny batches */
  if( max_inflight > 3UL ) max_inflight = 3UL;
  if( !*filling || inflight >= max_inflight ) return 0;
  /* throughput knob (opt.min_batch / max_wait_ns): a partial batch smaller than min_batch waits until
     its oldest frag has waited max_wait -- bigger GPU batches under load */
  if( *filling < vt->min_batch && now - vt->fill_t0 < vt->max_wait_ns ) return 0;
  if( vt->nctx > 1 && *filling < vt->batch ) {
    /* stagger: launch once every other context's newest batch has run
       batch_ns / nctx (or that context is idle) */
    ulong stagger = (ulong)( vt->batch_ns / (double)vt->nctx );
    for( int k=0; k<vt->nctx; k++ )
      if( k != f && vt->busy[k] && now - vt->launch_ns[k] < stagger ) return 0;
  }
  return 1;
}

int
fdgpu_vtile_housekeep( fdgpu_vtile_t * vt, ulong max_inflight ) {
  ulong filling, now = now_ns();
  vt_cp_publish( vt );                           /* copy tasks written since the last group of 16 */
  if( vt->svc ) {                                /* served: the service decides launches and copies */
    vt_svc_publish( vt );
    vt_copy_poll( vt );
    return 0;
  }
  /* batch duration: a context's batches have drained (inflight counts
     launched slots not yet fully polled) */
  for( int k=0; k<vt->nctx; k++ ) {
    if( !vt->busy[k] ) continue;
    ulong f, i;
    fdgpu_ed25519_pipeline_state( vt->ctx[k], &f, &i );
    if( !i ) {
      vt->busy[k] = 0; vt->batch_ns = 0.875*vt->batch_ns + 0.125*(double)( now - vt->launch_ns[k] );
    }
  }
  int f = vt->fill, launched = 0;
  if( vt_should_launch( vt, f, max_inflight, now, &filling ) ) {
    vt_fence();
    if( !fdgpu_ed25519_flush( vt->ctx[f] ) ) {   /* (the launch gathers the batch's frags not yet copied) */
      vt_launched( vt, f, now, filling );
      vt->fill = ( f + 1 ) % vt->nctx;
      vt->copy_t0 = 0UL;
      launched = 1;
    }
  } else if( vt->zc && vt->copy_t0 && !fdgpu_ed25519_faulted( vt->ctx[f] ) &&
             ( now - vt->copy_t0 >= vt->opt.copy_wait_ns ||
               vt->sub_cnt[f] - fdgpu_ed25519_gather_launched( vt->ctx[f] ) >= vt->opt.copy_min ) ) {
    /* the batch waits for the GPU: copy the frags taken since the last copy now, once the oldest has
       waited copy_wait_ns or copy_min are waiting -- what bounds a frag's exposure to a lapping
       producer (and a reliable link's credit) to about copy_wait_ns plus one gather, whatever the
       batch size and however long it queues */
    if( fdgpu_ed25519_gather( vt->ctx[f] ) > 0 ) vt_copy_launched( vt, f );
    vt->copy_t0 = 0UL;
  }
  vt_copy_poll( vt );
  return launched;
}

/* room for one more frag, and a healthy context to fill: 0, -2 (ring full: drain and retry), -3 */
static int
vt_room( fdgpu_vtile_t * vt ) {
  if( !vt->zc ) vt_fence();                      /* (zero-copy intake makes no streaming stores) */
  if( vt->pend_tail - vt->pend_head >= vt->pend_cap ) { fdgpu_vtile_flush( vt ); return -2; }
  if( vt->svc ) return 0;                        /* (a served tile's frags complete as faults if the service's batch fails) */
  /* a faulted context takes no more frags: fill the next healthy one (none: -3) */
  if( __builtin_expect( fdgpu_ed25519_faulted( vt->ctx[ vt->fill ] ), 0 ) ) {
    for( int i=0; i<vt->nctx && fdgpu_ed25519_faulted( vt->ctx[ vt->fill ] ); i++ ) vt->fill = ( vt->fill + 1 ) % vt->nctx;
    if( fdgpu_ed25519_faulted( vt->ctx[ vt->fill ] ) ) return -3;
  }
  return 0;
}

/* the frag whose record is (or will be, gathered) at the out dcache's out_chunk was submitted */
static void
vt_taken( fdgpu_vtile_t * vt, int in_idx, ulong seq, ulong tsorig, ulong bundle_id, unsigned short payload_sz ) {
  vt_pend_t * p = &vt->pend[ vt->pend_tail % vt->pend_cap ];
  p->seq = seq; p->tsorig = tsorig; p->chunk = vt->out_chunk; p->k = vt->fill; p->ovr = 0; p->in_idx = in_idx; p->cp = 0UL;
  if( vt->zc ) {
    p->cidx = vt->svc ? 0UL : vt->sub_cnt[ vt->fill ]++;
    vt->uncopied[ in_idx ]++; vt->uncopied_tot++;
    if( !vt->copy_t0 ) vt->copy_t0 = now_ns();
  }
  if( vt->min_batch && !vt->svc ) {                          /* first frag of the filling batch: its wait starts */
    ulong f, i; fdgpu_ed25519_pipeline_state( vt->ctx[ vt->fill ], &f, &i );
    if( f == 1UL ) vt->fill_t0 = now_ns();
  }
  p->bundle_id = bundle_id; p->payload_sz = payload_sz;
  vt->pend_tail++;
  ulong reserve = ( ( FDGPU_TXNM_HDR_SZ + payload_sz + 1UL ) & ~1UL ) + 852UL;
  vt->out_chunk = fdgpu_dcache_compact_next( vt->out_chunk, reserve, vt->chunk0, vt->wmark );
  if( vt->svc && vt->pend_tail - vt->req_pub >= 16UL ) vt_svc_publish( vt );   /* requests in groups of 16 */
}

/* submit the record the host has just written at dst (the out dcache's out_chunk) */
static int
vt_submit_host_record( fdgpu_vtile_t * vt, uchar * dst, unsigned short payload_sz, ulong seq ) {
  if( vt->svc ) {        /* served: the GPU reads the record where the tile wrote it (its out dcache) */
    vt_svc_req( vt, ( VSVC_RGN_OUT << 56 ) | (ulong)( dst - vt->dcache ), VSVC_LINE_NONE, seq, FDGPU_TXNM_HDR_SZ + payload_sz,
                VSVC_REQ_HOSTCOPY );
    return 0;
  }
  if( vt->zc )   /* keep the batch in gathered mode: the GPU "gathers" the record from where it already is */
    return fdgpu_ed25519_submit_raw_gather_chk( vt->ctx[ vt->fill ], dst, vt->dcache, dst,
                                                (unsigned short)( FDGPU_TXNM_HDR_SZ + payload_sz ),
                                                (unsigned short)FDGPU_TXNM_HDR_SZ, payload_sz, vt->pend_tail, NULL,
                                                seq );
  return fdgpu_ed25519_submit_raw_ref( vt->ctx[ vt->fill ], vt->dcache, dst + FDGPU_TXNM_HDR_SZ, payload_sz, vt->pend_tail );
}

static int vt_during_gossip( fdgpu_vtile_t * vt, int link, void const * frag, ulong sz, ulong readable, ulong seq,
                             ulong tsorig );

/* during_frag of an fd_txn_m_t record (QUIC, bundle and send in links).  readable: bytes readable from frag
   (its sz for a frag given by pointer; the link's MTU on the chunk path) */
static int
vt_during_txnm( fdgpu_vtile_t * vt, int link, void const * frag, ulong sz, ulong readable, ulong seq, ulong tsorig ) {
  fdgpu_txnm_t const * in = (fdgpu_txnm_t const *)frag;
  /* fd_verify_tile.c:75-85: the frag fits FD_TPU_RAW_MTU and the payload fits the MTU (the reference
     FD_LOG_ERRs).  The reference does not check the payload against sz: a frag whose header the producer
     was rewriting while the stem read its line (a lapped consumer) may claim more than sz, and the stem's
     seq re-check then drops it.  So on the chunk path a payload past sz is taken (its bytes lie in the
     link's region; the stem's check, or the GPU copy's, marks the frag overrun); by pointer, where only the
     frag's sz bytes are known readable, it is corrupt.  Only that overrun case matches the reference: a frag
     NOT lapped whose header claims a payload past sz is copied here as 80 + payload_sz bytes of the in link
     (the bytes after the frag), where the reference copies sz bytes (fd_verify_tile.c:79) and parses the rest
     from whatever its out dcache held there before -- stale memory, so the two verdicts may differ for such a
     malformed producer (parity unpinned in that corner; no test covers it). */
  if( sz > FDGPU_TPU_RAW_MTU || sz < FDGPU_TXNM_HDR_SZ || in->payload_sz > 1232U ||
      FDGPU_TXNM_HDR_SZ + in->payload_sz > readable )
    return -4;
  if( vt->zc && link >= vt->n_in ) return -4;            /* a link the zero-copy intake was not told about */
  int rc = vt_room( vt );
  if( rc ) return rc;
  if( vt->zc && vt->uncopied_tot >= vt->opt.max_uncopied ) {   /* copy backlog: start the copies, take nothing */
    vt_copy_poll( vt );
    if( vt->uncopied_tot >= vt->opt.max_uncopied ) {
      if( vt->svc ) { vt_svc_publish( vt ); atomic_fetch_add_explicit( &vt->sc->gather, 1UL, memory_order_release ); }
      for( int k=0; k<vt->nctx; k++ )
        if( !fdgpu_ed25519_faulted( vt->ctx[k] ) && fdgpu_ed25519_gather( vt->ctx[k] ) > 0 ) vt_copy_launched( vt, k );
      vt->copy_t0 = 0UL;
      vt->gm.copy_backlog++;
      return FDGPU_VTILE_COPY_BACKLOG;
    }
  }
  uchar * dst = vt->dcache + vt->out_chunk * FDGPU_CHUNK_SZ;
  if( vt->zc && vt->svc ) {   /* served: the request names the frag's and its line's places in the service's regions */
    fdgpu_mcache_t const * mc = vt->in_mcs[ link ];
    ulong rsz = FDGPU_TXNM_HDR_SZ + in->payload_sz;
    ulong src = vt_svc_ref( vt, frag, ( rsz + 15UL ) & ~15UL );
    if( src == ~0UL || ( (ulong)frag & 15UL ) ) return -3;            /* not in a region of the service */
    ulong line = VSVC_LINE_NONE;
    if( mc ) line = vt->in_line_ref[ link ] + ( seq & ( mc->depth - 1UL ) ) * sizeof(mc_line_t);
    vt_svc_req( vt, src, line, seq, rsz, vt->ncp ? VSVC_REQ_HOSTCOPY : 0U );
    vt_taken( vt, link, seq, tsorig, in->bundle_id, in->payload_sz );
    if( vt->ncp ) {            /* the record's copy into the out dcache: one of the tile's copy threads */
      vt_pend_t * p = &vt->pend[ ( vt->pend_tail - 1UL ) % vt->pend_cap ];
      ulong i = vt->cp_cnt++;
      vt_cp_t * cq = vt->cp[ i % (ulong)vt->ncp ];
      ulong t = cq->ptail;
      vt_cp_task_t * k = &cq->ring[ t & cq->mask ];
      k->src = (uchar const *)frag; k->dst = dst; k->sz = rsz;
      k->line_seq = mc ? (ulong const *)&mc->line[ seq & ( mc->depth - 1UL ) ].seq : NULL; k->seq = seq; k->ovr = &p->ovr;
      cq->ptail = t + 1UL;
      if( !( cq->ptail & 15UL ) ) atomic_store_explicit( &cq->tail, cq->ptail, memory_order_release );
      p->cp = i + 1UL;
    }
    return 0;
  }
  if( vt->zc ) {   /* the GPU copies the frag into dst itself (no host copy) and re-checks its mcache line */
    fdgpu_mcache_t const * mc = vt->in_mcs[ link ];
    /* device views: the mcache lines' translated once (set_in_links), the frag's region cached */
    ulong const * seq_dev = NULL;
    if( mc ) {
      if( !vt->in_mc_dev[ link ] ) return -3;
      ulong li = seq & ( mc->depth - 1UL );
      seq_dev = (ulong const *)( vt->in_mc_dev[ link ] + ( (uchar const *)&mc->line[ li ].seq - (uchar const *)mc->line ) );
    }
    uchar const * src = (uchar const *)frag;
    ulong csz = ( FDGPU_TXNM_HDR_SZ + in->payload_sz + 15UL ) & ~15UL;
    if( src < vt->src_lo || src + csz > vt->src_hi ) {
      void * b, * d; ulong rs;
      if( fdgpu_host_region( src, &b, &rs, &d ) ) return -3;   /* not in a registered region */
      vt->src_lo = (uchar const *)b; vt->src_hi = (uchar const *)b + rs; vt->src_dev = (uchar const *)d;
      if( src + csz > vt->src_hi ) return -3;
    }
    rc = fdgpu_ed25519_submit_raw_gather_dev_f( vt->ctx[ vt->fill ], src, vt->src_dev + ( src - vt->src_lo ), vt->dcache, dst,
                                                (unsigned short)( FDGPU_TXNM_HDR_SZ + in->payload_sz ),
                                                (unsigned short)FDGPU_TXNM_HDR_SZ, in->payload_sz, vt->pend_tail,
                                                seq_dev, seq, vt->ncp ? FDGPU_GATHER_NO_WRITEBACK : 0U );
    if( rc ) return rc;
    vt_taken( vt, link, seq, tsorig, in->bundle_id, in->payload_sz );
    if( vt->ncp ) {            /* the record's copy into the out dcache: one of the tile's copy threads */
      vt_pend_t * p = &vt->pend[ ( vt->pend_tail - 1UL ) % vt->pend_cap ];
      ulong i = vt->cp_cnt++;
      vt_cp_t * cq = vt->cp[ i % (ulong)vt->ncp ];
      ulong t = cq->ptail;
      vt_cp_task_t * k = &cq->ring[ t & cq->mask ];
      k->src = src; k->dst = dst; k->sz = FDGPU_TXNM_HDR_SZ + in->payload_sz;
      k->line_seq = mc ? (ulong const *)&mc->line[ seq & ( mc->depth - 1UL ) ].seq : NULL; k->seq = seq; k->ovr = &p->ovr;
      cq->ptail = t + 1UL;
      if( !( cq->ptail & 15UL ) ) atomic_store_explicit( &cq->tail, cq->ptail, memory_order_release );
      p->cp = i + 1UL;
    }
    return 0;
  } else {
    vt_copy( dst, (uchar const *)frag, FDGPU_TXNM_HDR_SZ + in->payload_sz );
    rc = vt_submit_host_record( vt, dst, in->payload_sz, seq );
  }
  if( rc ) return rc;
  vt_taken( vt, link, seq, tsorig, in->bundle_id, in->payload_sz );
  return 0;
}

int
fdgpu_vtile_during_frag( fdgpu_vtile_t * vt, ulong in_idx, void const * frag, ulong sz, ulong seq, ulong tsorig ) {
  if( in_idx >= FDGPU_VTILE_IN_MAX ) return -4;
  /* a frag given by pointer: only its sz bytes are known to be readable */
  if( vt->in_kind[ in_idx ] == FDGPU_VTILE_IN_KIND_GOSSIP ) return vt_during_gossip( vt, (int)in_idx, frag, sz, sz, seq, tsorig );
  return vt_during_txnm( vt, (int)in_idx, frag, sz, sz, seq, tsorig );
}

int
fdgpu_vtile_during_frag_chunk( fdgpu_vtile_t * vt, ulong in_idx, ulong seq, ulong sig, ulong chunk, ulong sz, ulong ctl,
                               ulong tsorig ) {
  (void)sig; (void)ctl;
  if( in_idx >= FDGPU_VTILE_IN_MAX || !vt->in_mem[ in_idx ] ) return -4;
  /* fd_verify_tile.c:75-76,89-90: a chunk outside the link's [chunk0, wmark] is corrupt (FD_LOG_ERR) */
  if( chunk < vt->in_chunk0[ in_idx ] || chunk > vt->in_wmark[ in_idx ] ) return -4;
  uchar const * frag = vt->in_mem[ in_idx ] + chunk * FDGPU_CHUNK_SZ;
  /* a gossip frame inside its link's dcache: the region holds FDGPU_GOSSIP_MSG_MAX bytes from any chunk up to
     wmark (fdgpu_vtile_set_in), so vote.txn's whole 1232-byte array is readable past a shorter frame, as the
     reference reads it (fd_verify_tile.c:91-95) */
  if( vt->in_kind[ in_idx ] == FDGPU_VTILE_IN_KIND_GOSSIP )
    return vt_during_gossip( vt, (int)in_idx, frag, sz, FDGPU_GOSSIP_MSG_MAX, seq, tsorig );
  return vt_during_txnm( vt, (int)in_idx, frag, sz, FDGPU_TPU_RAW_MTU, seq, tsorig );
}

int
fdgpu_vtile_set_in( fdgpu_vtile_t * vt, ulong in_idx, int in_kind, void const * mem, ulong chunk0, ulong wmark ) {
  if( in_idx >= FDGPU_VTILE_IN_MAX || in_kind < FDGPU_VTILE_IN_KIND_QUIC || in_kind > FDGPU_VTILE_IN_KIND_SEND ) return -1;
  if( vt->pend_tail != vt->pend_head ) return -1;       /* only while idle */
  vt->in_kind[ in_idx ] = in_kind;
  vt->in_mem[ in_idx ] = (uchar const *)mem; vt->in_chunk0[ in_idx ] = chunk0; vt->in_wmark[ in_idx ] = wmark;
  return 0;
}

/* The reference's other in kinds (fd_verify_tile.c:7-10).  before_frag
   (:36-59): a QUIC frag, or a bundle-tile "packet" (sig 0), goes to the
   tile with seq % round_robin_cnt == its index; a bundle (sig != 0) only
   to verify:0, so a bundle's transactions are never interleaved across
   tiles; a gossip update only if it is a vote (sig ==
   FD_GOSSIP_UPDATE_TAG_VOTE) and round robin; a send-tile frag always. */
void
fdgpu_vtile_set_round_robin( fdgpu_vtile_t * vt, ulong idx, ulong cnt ) {
  vt->rr_cnt = cnt ? cnt : 1UL; vt->rr_idx = idx < vt->rr_cnt ? idx : 0UL;
}

int
fdgpu_vtile_before_frag( fdgpu_vtile_t const * vt, ulong in_idx, ulong seq, ulong sig ) {
  if( in_idx >= FDGPU_VTILE_IN_MAX ) return 1;
  int in_kind = vt->in_kind[ in_idx ];
  ulong cnt = vt->rr_cnt ? vt->rr_cnt : 1UL;
  int is_bundle_packet = in_kind==FDGPU_VTILE_IN_KIND_BUNDLE && !sig;
  if( is_bundle_packet || in_kind==FDGPU_VTILE_IN_KIND_QUIC ) return ( seq % cnt ) != vt->rr_idx;
  if( in_kind==FDGPU_VTILE_IN_KIND_BUNDLE ) return vt->rr_idx != 0UL;
  if( in_kind==FDGPU_VTILE_IN_KIND_GOSSIP ) return ( seq % cnt ) != vt->rr_idx || sig != FDGPU_GOSSIP_UPDATE_TAG_VOTE;
  return 0;
}

/* during_frag of every in kind (:65-101).  QUIC, bundle and send frags are
   fd_txn_m_t records (fdgpu_vtile_during_frag).  A gossip frag is an
   fd_gossip_update_message_t: its vote transaction becomes a fresh
   record in the out dcache -- payload_sz, bundle_id 0, the payload -- as
   the reference copies it; the GPU takes it from there (the gossip link
   is reliable in the reference topology, topology.c:591, so there is no
   overrun to check).  The reference leaves the record's other header
   fields as the chunk's previous frag left them; here they are zero. */
static int
vt_during_gossip( fdgpu_vtile_t * vt, int link, void const * frag, ulong sz, ulong readable, ulong seq, ulong tsorig ) {
  if( sz > FDGPU_GOSSIP_MSG_MAX || sz < FDGPU_GOSSIP_VOTE_TXN_OFF ) return -4;   /* :89-90 */
  uchar const * msg = (uchar const *)frag;
  ulong txn_sz; memcpy( &txn_sz, msg + FDGPU_GOSSIP_VOTE_TXN_SZ_OFF, sizeof(ulong) );
  /* the reference copies vote.txn_sz bytes out of the 1232-byte vote.txn array unchecked
     (fd_verify_tile.c:91-95), also past the frame the gossip tile publishes (FD_GOSSIP_UPDATE_SZ_VOTE
     = 1297 bytes ends 1225 bytes into vote.txn, fd_gossip_private.h:80): so does this where the bytes
     are known to be readable (`readable` from frag: the link's dcache on the chunk path, the frame
     itself for a frag given by pointer).  Past the array there is nothing defined to copy: refused as
     corrupt, as is a vote that would be read past the readable bytes */
  if( txn_sz > 1232UL || FDGPU_GOSSIP_VOTE_TXN_OFF + txn_sz > readable ) return -4;
  int rc = vt_room( vt );
  if( rc ) return rc;
  uchar * dst = vt->dcache + vt->out_chunk * FDGPU_CHUNK_SZ;
  fdgpu_txnm_t * t = (fdgpu_txnm_t *)dst;
  memset( t, 0, FDGPU_TXNM_HDR_SZ );
  t->payload_sz = (unsigned short)txn_sz;
  t->bundle_id = 0UL;
  memcpy( dst + FDGPU_TXNM_HDR_SZ, msg + FDGPU_GOSSIP_VOTE_TXN_OFF, txn_sz );
  vt_fence();
  rc = vt_submit_host_record( vt, dst, (unsigned short)txn_sz, seq );
  if( rc ) return rc;
  vt_taken( vt, link, seq, tsorig, 0UL, (unsigned short)txn_sz );
  return 0;
}

int
fdgpu_vtile_during_frag_overrun( fdgpu_vtile_t * vt ) {
  if( vt->pend_tail == vt->pend_head ) return -1;
  vt->pend[ ( vt->pend_tail - 1UL ) % vt->pend_cap ].ovr = 1;
  return 0;
}

/* after_frag (fd_verify_tile.c:103-157) for one completed frag.  The GPU
   returned the code, the footprint and the dedup tag; with zero-copy intake
   it also wrote the record (payload, txn_t_sz, fd_txn_t image) into the out
   dcache, so this touches only the tcache and, for the overrun check, the
   in mcache line. */
static int
vt_after( fdgpu_vtile_t * vt, vt_pend_t const * p, int code, uchar const * img, unsigned fp, ulong tag,
          fdgpu_vtile_done_t * d ) {
  d->seq = p->seq; d->in_idx = (ulong)p->in_idx; d->tsorig = p->tsorig; d->chunk = p->chunk; d->sz = 0UL; d->tag = 0UL;
  d->code = code;
  /* zero-copy: the GPU re-read the frag's mcache line right after copying it and found it reused
     -- the stem's "overrun while reading" (fd_stem.c:667-686), decided at copy time: the frag
     never reaches after_frag in the reference, so no bundle state or metric changes */
  if( code == FDGPU_ERR_OVERRUN || p->ovr ) { vt->overruns++; return FDGPU_VTILE_OVERRUN; }
  fdgpu_txnm_t * txnm = (fdgpu_txnm_t *)( vt->dcache + p->chunk * FDGPU_CHUNK_SZ );
  if( !vt->gpu_rec ) txnm->txn_t_sz = (unsigned short)fp;
  int is_bundle = p->bundle_id != 0UL;
  if( is_bundle && p->bundle_id != vt->bundle_id ) { vt->bundle_failed = 0; vt->bundle_id = p->bundle_id; }
  if( is_bundle && vt->bundle_failed ) { vt->metrics[3]++; return FDGPU_VTILE_BUNDLE_PEER_FAIL; }
  if( code == FDGPU_ERR_PARSE ) {
    if( is_bundle ) vt->bundle_failed = 1;
    vt->metrics[0]++;
    return FDGPU_VTILE_PARSE_FAIL;
  }
  if( !vt->gpu_tag ) {        /* host XXH64 of the first signature (A/B knob; reads payload and image) */
    uchar const * payload = (uchar const *)txnm + FDGPU_TXNM_HDR_SZ;
    uchar const * im = vt->gpu_rec ? (uchar const *)txnm + ( ( FDGPU_TXNM_HDR_SZ + p->payload_sz + 1UL ) & ~1UL ) : img;
    tag = xxh64_64( vt->seed, payload + ( (unsigned)im[2] | ((unsigned)im[3] << 8) ) );
  }
  /* fd_txn_verify (fd_verify_tile.h:59-108): dedup query, verify, insert */
  int res = 0;   /* 0 success, 1 verify failed, 2 dedup */
  if( !is_bundle ) {             /* query; a verified tag goes in at the slot the query's probe found */
    if( tc_query_insert( vt->tcache, tag, code == 0 ) ) res = 2;
    else if( code != 0 ) res = 1;
  } else if( code != 0 ) res = 1;
  if( res ) {
    if( is_bundle ) vt->bundle_failed = 1;
    if( res==2 ) { vt->metrics[2]++; return FDGPU_VTILE_DEDUP_FAIL; }
    vt->metrics[1]++;
    return FDGPU_VTILE_VERIFY_FAIL;
  }
  /* publish: fd_txn_t behind the payload at a 2-byte boundary */
  ulong t_off = ( FDGPU_TXNM_HDR_SZ + p->payload_sz + 1UL ) & ~1UL;
  if( !vt->gpu_rec ) memcpy( (uchar *)txnm + t_off, img, fp );
  d->sz = t_off + fp;                                  /* fd_txn_m_realized_footprint( txnm, 1, 0 ) */
  d->tag = is_bundle ? 0UL : tag;
  vt->metrics[4]++;
  return FDGPU_VTILE_PUBLISH;
}

/* the frag at the head leaves the pending ring (a verdict implies its copy completed) */
static inline void vt_pop( fdgpu_vtile_t * vt, vt_pend_t const * p ) {
  if( vt->zc && vt->copy_cursor == vt->pend_head ) { vt_copied( vt, p ); vt->copy_cursor++; }
  vt->pend_head++;
}

/* after_frags of a served tile: the service's completions, in request (= pending) order */
static ulong
vt_after_frags_svc( fdgpu_vtile_t * vt, fdgpu_vtile_done_t * out, ulong max, int blocking ) {
  ulong n = 0UL;
  vsvc_client_t * sc = vt->sc;
  vt_cp_publish( vt );
  vt_svc_publish( vt );
  if( blocking ) atomic_fetch_add_explicit( &sc->flush, 1UL, memory_order_release );   /* never wait on an unlaunched batch */
  while( n < max && vt->pend_head < vt->pend_tail ) {
    ulong tw = now_ns();
    ulong tail = atomic_load_explicit( &sc->cpl_tail, memory_order_acquire );
    if( tail == vt->cpl_seen ) {
      if( vt_svc_dead( vt ) ) {
        /* the service is gone: no verdict will come.  The pending frags complete, in order, as
           FDGPU_VTILE_GPU_FAULT (never published, never blocked on), as a faulted context's do */
        while( n < max && vt->pend_head < vt->pend_tail ) {
          vt_pend_t const * p = &vt->pend[ vt->pend_head % vt->pend_cap ];
          vt_cp_wait( vt, p );
          fdgpu_vtile_done_t * d = &out[n];
          d->seq = p->seq; d->in_idx = (ulong)p->in_idx; d->tsorig = p->tsorig; d->chunk = p->chunk; d->sz = 0UL; d->tag = 0UL;
          d->result = FDGPU_VTILE_GPU_FAULT; d->code = 0; d->ctx = 255U; d->batch_txns = 0U; d->batch_pos = 0U;
          d->path = FDGPU_PATH_NONE;
          vt->gm.gpu_fault_frags++;
          vt_pop( vt, p ); n++;
        }
        break;
      }
      if( !blocking ) break;
      ulong t_spin = now_ns();
      while( atomic_load_explicit( &sc->cpl_tail, memory_order_acquire ) == vt->cpl_seen && now_ns() - t_spin < 1000000UL )
        _mm_pause();
      vt->gm.wait_ns += now_ns() - tw;
      continue;
    }
    ulong tp = now_ns();
    vt->gm.poll_ns += tp - tw;
    ulong k = tail - vt->cpl_seen;
    if( k > max - n ) k = max - n;
    for( ulong i=0; i<k; i++ ) {
      vsvc_cpl_t const * c = &vt->scpl[ vt->cpl_seen & vt->smask ];
      if( c->req != (unsigned)vt->pend_head ) {   /* completions come back in request order */
        fprintf( stderr, "fdgpu_vtile_after_frags: service completion %u != pending frag %lu\n", c->req, vt->pend_head );
        abort();
      }
      if( i + 8UL < k && vt->gpu_tag ) tc_prefetch( vt->tcache, vt->scpl[ ( vt->cpl_seen + 8UL ) & vt->smask ].dtag, 8UL );
      vt_pend_t const * p = &vt->pend[ vt->pend_head % vt->pend_cap ];
      vt_cp_wait( vt, p );
      fdgpu_vtile_done_t * d = &out[n];
      if( c->code == VSVC_CODE_FAULT ) {               /* its batch failed in the service: no verdict */
        d->seq = p->seq; d->in_idx = (ulong)p->in_idx; d->tsorig = p->tsorig; d->chunk = p->chunk; d->sz = 0UL; d->tag = 0UL;
        d->result = FDGPU_VTILE_GPU_FAULT; d->code = 0;
        vt->gm.gpu_fault_frags++;
      } else {
        d->result = vt_after( vt, p, (int)c->code, NULL, c->fp, c->dtag, d );
      }
      d->ctx = c->ctx; d->batch_txns = c->batch_txns; d->batch_pos = c->batch_pos; d->path = c->path;
      vt_pop( vt, p ); n++;
      vt->cpl_seen++;
    }
    vt->gm.after_ns += now_ns() - tp;
    blocking = 0;
  }
  return n;
}

ulong
fdgpu_vtile_after_frags( fdgpu_vtile_t * vt, fdgpu_vtile_done_t * out, ulong max, int blocking ) {
  if( vt->svc ) return vt_after_frags_svc( vt, out, max, blocking );
  ulong n = 0UL;
  if( blocking ) fdgpu_vtile_flush( vt );      /* a blocking drain must not wait on an unlaunched batch */
  while( n < max && vt->pend_head < vt->pend_tail ) {
    /* the next completions in frag order: the run of pending frags from
       the head that went to the same context (each context completes in
       its own submission order) */
    int c = vt->pend[ vt->pend_head % vt->pend_cap ].k;
    ulong want, lim = max - n;
    if( fdgpu_ed25519_faulted( vt->ctx[c] ) ) {
      want = 1UL;
      while( want < lim && vt->pend_head + want < vt->pend_tail &&
             vt->pend[ ( vt->pend_head + want ) % vt->pend_cap ].k == c ) want++;
      /* the context's batches failed on the device: its frags will never get a
         verdict.  Complete them, in order, as FDGPU_VTILE_GPU_FAULT (never
         published, never blocked on); the caller treats that as the
         reference's FD_LOG_ERR or recreates the context (fdgpu_vtile_recover). */
      if( !vt->fault_seen[c] ) { vt->fault_seen[c] = 1; vt->gm.faults++; }
      for( ulong i=0; i<want; i++ ) {
        vt_pend_t const * p = &vt->pend[ vt->pend_head % vt->pend_cap ];
        vt_cp_wait( vt, p );                   /* (its copy thread writes the entry's ovr: not reused before) */
        fdgpu_vtile_done_t * d = &out[n];
        d->seq = p->seq; d->in_idx = (ulong)p->in_idx; d->tsorig = p->tsorig; d->chunk = p->chunk; d->sz = 0UL; d->tag = 0UL;
        d->result = FDGPU_VTILE_GPU_FAULT; d->code = 0;
        d->ctx = (unsigned)c; d->batch_txns = 0U; d->batch_pos = 0U; d->path = FDGPU_PATH_NONE;
        vt->gm.gpu_fault_frags++;
        vt_pop( vt, p ); n++;
      }
      continue;
    }
    /* the frag at the head is the next verdict of context c's oldest launched batch, whose
       frags are contiguous in the pending ring: poll at most what that batch has left (0: the
       head frag's batch is still filling) */
    want = fdgpu_ed25519_front_remaining( vt->ctx[c] );
    if( want > lim ) want = lim;
    if( !want ) break;                         /* (a blocking call launched every filling batch above) */
    ulong b_txns, b_cur; int b_path;              /* the batch these verdicts come from (diagnostics) */
    fdgpu_ed25519_front_batch( vt->ctx[c], &b_txns, &b_cur, &b_path );
    ulong tw = now_ns();
    ulong k = fdgpu_ed25519_poll_raw( vt->ctx[c], vt->p_tags, vt->p_codes, vt->zc ? NULL : vt->p_img, vt->p_fp, vt->p_dtag,
                                      want, blocking );
    ulong tp = now_ns();
    if( blocking ) vt->gm.wait_ns += tp - tw; else vt->gm.poll_ns += tp - tw;
    if( !k ) {
      if( fdgpu_ed25519_faulted( vt->ctx[c] ) ) continue;   /* failed just now: complete its frags above */
      break;
    }
    for( ulong i=0; i<k; i++ ) {
      if( vt->p_tags[i] != vt->pend_head ) {   /* completions must come back in submission order */
        fprintf( stderr, "fdgpu_vtile_after_frags: completion tag %lu != pending frag %lu\n", vt->p_tags[i], vt->pend_head );
        abort();
      }
      /* the random accesses of after_frag are the tcache map slots (of this tag, and of the
         tag the insert evicts) and, with an in link, the frag's mcache line: start them a
         few completions ahead */
      if( i + 8UL < k && vt->gpu_tag ) tc_prefetch( vt->tcache, vt->p_dtag[ i + 8UL ], 8UL );
      if( !vt->zc && vt->pend_head + 4UL < vt->pend_tail ) {   /* host-copied records: the header line */
        uchar * r = vt->dcache + vt->pend[ ( vt->pend_head + 4UL ) % vt->pend_cap ].chunk * FDGPU_CHUNK_SZ;
        __builtin_prefetch( r, 1 );
      }
      vt_pend_t const * p = &vt->pend[ vt->pend_head % vt->pend_cap ];
      vt_cp_wait( vt, p );                     /* the record's host copy and its line re-check (copy threads) */
      /* tags are the pending counter: completions come back in order */
      out[n].result = vt_after( vt, p, (int)vt->p_codes[i], vt->p_img + i*FDGPU_TXN_IMG_STRIDE, vt->p_fp[i],
                                vt->p_dtag[i], &out[n] );
      out[n].ctx = (unsigned)c; out[n].batch_txns = (unsigned)b_txns; out[n].batch_pos = (unsigned)( b_cur + i );
      out[n].path = b_path;
      vt_pop( vt, p ); n++;
    }
    vt->gm.after_ns += now_ns() - tp;
    blocking = 0;
  }
  return n;
}

/* ---- the configs[4] stream: Q producer links, T verify tiles -----------
   The reference wires the verify stage as one out link per QUIC tile, each
   read by every verify tile: tile i takes the frags with seq % T == i of
   every link (before_frag, fd_verify_tile.c:47-48; topology.c:167-169) over
   UNRELIABLE, overrunnable links.  Here the links -- Q mcaches, one in
   dcache prefilled with one fd_txn_m_t record per distinct payload (what
   QUIC reassembly leaves; producer q's frag s points at payload
   (s Q + q) % n_payload), the per-link per-tile fseqs and the per-tile
   results -- are one memory region: a shared file (/dev/shm) when the tiles
   live in several processes (one per GPU; tile i drives GPU i % G, so
   process g runs the tiles i % G == g and the producers q % G == g), or
   private memory for a single process.  The producers (threads) stand in
   for the QUIC tiles: their timed loops only publish metadata.  Reliable
   links (credit based: a producer stays depth/2 ahead of the slowest tile
   on its link) lose nothing; unreliable ones never wait and a tile that
   falls a lap behind on a link is overrun: it resumes at the seq it found
   (fd_stem.c:590-596, 676-688) and the frags it skipped are counted.  A
   frag goes to during_frag with its link as in_idx and its own seq. */

#define LINK_MAGIC    0xfd6e11c0ffee0004UL
#define LINK_TILE_MAX 64
#define LINK_ANOM_MAX 8

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

typedef struct {                 /* one tile's results, written once when it finishes */
  ulong verdicts;                /* own frags returned by after_frags (any result) */
  ulong lost;                    /* own frags skipped by polling / reading overruns (unreliable link) */
  ulong overruns;                /* of the verdicts: FDGPU_VTILE_OVERRUN (overwritten before the GPU read it) */
  ulong sigs, t_last, lmax;
  ulong metrics[5];
  ulong ns[4];                   /* during_frag intake (mcache polls + submit), after_frags, housekeep, whole loop */
  ulong ns_idle;                 /* of ns[0]: intake passes that found nothing published */
  ulong prof[ 8 ];               /* FDGPU_LINK_PROF=1: section times, ns (fdgpu_stream_stats_t prof_ns) */
  fdgpu_vtile_gpu_metrics_t gm;
  ulong device;
  ulong cpu_ns, wall_ns, nivcsw; /* the tile thread's CPU time over its loop's wall time, involuntary switches */
  long  cpu;                     /* the CPU it was pinned to (-1: none) */
  /* written as the tile runs (fdgpu_link_trace / fdgpu_link_anomalies): its verdicts traced so far, and the first
     LINK_ANOM_MAX verdicts that were neither published nor overrun (parse / verify / dedup / bundle failures)
     with how many there were -- in the link, so a tile in a process of its own (served tiles) reports them too */
  ulong trace_cnt;
  ulong anom_cnt;
  ulong anom_by_result[ 8 ];     /* those verdicts by result (FDGPU_VTILE_*); [0]: dedups of payloads the tile published before */
  ulong gpu_open;                /* the tile's process had the GPU open (/dev/kfd, /dev/dri) when it finished */
  fdgpu_link_anomaly_t anom[ LINK_ANOM_MAX ];
} link_res_t;

#define LINK_PROD_MAX FDGPU_VTILE_IN_MAX


typedef struct {
  _Atomic ulong magic;           /* set last by the creator (release) */
  ulong         total_sz;
  fdgpu_stream_cfg_t cfg;        /* (cfg.producers normalised to 1..LINK_PROD_MAX) */
  ulong         depth, n_payload, in_bytes;
  ulong         off_mcache[ LINK_PROD_MAX ], off_dcache, off_chunk, off_sz, off_psig, off_res, off_hist, off_trace;
  _Atomic ulong joined, tiles_ready, tiles_done, go, fail;
  ulong         t_start;
  ulong         prod_end[ LINK_PROD_MAX ], prod_wait_ns[ LINK_PROD_MAX ];   /* per producer: last publish, credit waits */
  ulong         prod_cpu_ns[ LINK_PROD_MAX ], prod_wall_ns[ LINK_PROD_MAX ], prod_nivcsw[ LINK_PROD_MAX ];
  long          prod_cpu[ LINK_PROD_MAX ];     /* the CPU each producer was pinned to (-1: none) */
  struct { _Atomic ulong v; uchar pad[56]; } fseq[ LINK_PROD_MAX ][ LINK_TILE_MAX ];   /* per link: next seq each tile may lose */
  ulong         part_off[ LINK_PROD_MAX + 1 ];   /* the in dcache in per-producer parts (2 MiB aligned), from its start */
  int           dc_node[ LINK_PROD_MAX ], mc_node[ LINK_PROD_MAX ];   /* NUMA node each part / mcache's first page got */
} link_hdr_t;

struct fdgpu_link {
  link_hdr_t *     h;
  uchar *          base;
  ulong            sz;
  uchar *          map;          /* the mapping base is inside (private links: 2 MiB aligned within it) */
  ulong            map_sz;
  int              shared, registered;
  mc_line_t *      line[ LINK_PROD_MAX ];
  uchar *          dcache;
  unsigned *       chunk;
  unsigned short * psz;
  uchar *          psig;         /* signatures of each payload (the first byte), for the stream's sigs/s */
  link_res_t *     res;
  ulong *          hist;
  fdgpu_mcache_t   mc[ LINK_PROD_MAX ];   /* local views of the shared lines (the tiles' in links) */
  fdgpu_link_trace_t * trace[ LINK_TILE_MAX ];   /* the tiles' verdicts, in order: this process's own arrays
                                                    (fdgpu_link_set_trace) or the link's (cfg.trace_cap) */
  ulong            trace_cap;
  int              trace_own;
  char             path[ 256 ];                   /* a shared link's file ("" for private memory) */
  fdgpu_vsvc_stats_t svc_stats;                   /* served tiles: this process's service, after fdgpu_link_run */
  int              svc_cpu;
};

static ulong al64( ulong x ) { return ( x + 63UL ) & ~63UL; }

static void link_view( fdgpu_link_t * l ) {
  link_hdr_t * h = l->h;
  for( int q=0; q<h->cfg.producers; q++ ) {
    l->line[q] = (mc_line_t *)( l->base + h->off_mcache[q] );
    l->mc[q].depth = h->depth; l->mc[q].line = l->line[q]; l->mc[q].own = 0;
  }
  l->dcache = l->base + h->off_dcache;
  l->chunk  = (unsigned *)( l->base + h->off_chunk );
  l->psz    = (unsigned short *)( l->base + h->off_sz );
  l->psig   = l->base + h->off_psig;
  l->res    = (link_res_t *)( l->base + h->off_res );
  l->hist   = (ulong *)( l->base + h->off_hist );
  if( h->cfg.trace_cap ) {                       /* the tiles' traces in the link itself (any process may run a tile) */
    l->trace_cap = h->cfg.trace_cap; l->trace_own = 0;
    for( int i=0; i<h->cfg.tiles && i<LINK_TILE_MAX; i++ )
      l->trace[i] = (fdgpu_link_trace_t *)( l->base + h->off_trace ) + (ulong)i * h->cfg.trace_cap;
  }
}

/* frags producer q of Q publishes: n / Q, the first n % Q producers one more */
static ulong prod_frags( ulong n, ulong Q, ulong q ) { return n / Q + ( q < n % Q ? 1UL : 0UL ); }

/* NUMA placement of the link's memory without libnuma: the mbind / get_mempolicy system calls (MPOL_BIND of a
   range before its first touch; the node a touched page got) */
#define LINK_MPOL_BIND   2
#define LINK_MPOL_F_NODE (1<<0)
#define LINK_MPOL_F_ADDR (1<<1)
static void link_bind( void * p, ulong sz, int node ) {
  if( node < 0 || node >= 1024 ) return;
  ulong mask[ 16 ] = { 0 };
  mask[ node / 64 ] = 1UL << ( node % 64 );
  ulong lo = (ulong)p & ~4095UL, hi = ( (ulong)p + sz + 4095UL ) & ~4095UL;
  (void)syscall( SYS_mbind, lo, hi - lo, LINK_MPOL_BIND, mask, 1025UL, 0U );   /* (refused: first touch decides) */
}
static int link_node_of( void const * p ) {
  int node = -1;
  if( syscall( SYS_get_mempolicy, &node, NULL, 0UL, p, LINK_MPOL_F_NODE | LINK_MPOL_F_ADDR ) ) return -1;
  return node;
}
/* a CPU of node `node` this thread may run on (-1: none) */
static int node_cpu( int node ) {
  if( node < 0 ) return -1;
  char path[ 96 ]; snprintf( path, sizeof(path), "/sys/devices/system/node/node%d/cpulist", node );
  static __thread uchar set[ 1024 ];
  memset( set, 0, sizeof(set) );
  FILE * f = fopen( path, "r" );
  if( !f ) return -1;
  char buf[ 4096 ]; size_t n = fread( buf, 1, sizeof(buf)-1, f ); fclose( f ); buf[n] = 0;
  cpu_set_t aff; CPU_ZERO( &aff );
  if( sched_getaffinity( 0, sizeof(aff), &aff ) ) return -1;
  char * c = buf;
  while( *c ) {
    char * e; long a = strtol( c, &e, 10 ), b = a;
    if( e == c ) break;
    if( *e == '-' ) { c = e + 1; b = strtol( c, &e, 10 ); }
    for( long i=a; i<=b && i<1024; i++ ) if( i >= 0 && CPU_ISSET( (int)i, &aff ) ) return (int)i;
    c = e; if( *c == ',' ) c++; else break;
  }
  return -1;
}

typedef struct {
  fdgpu_link_t * l; int q, Q, node; ulong depth;
  uchar const * payload; unsigned const * off; unsigned short const * sz; ulong n_payload;
} link_fill_arg_t;

static void * link_fill( void * _a ) {
  link_fill_arg_t * a = (link_fill_arg_t *)_a;
  fdgpu_link_t * l = a->l;
  link_hdr_t * h = l->h;
  ulong q = (ulong)a->q, Q = (ulong)a->Q;
  uchar * part = l->dcache + h->part_off[q];
  ulong part_sz = h->part_off[q+1] - h->part_off[q];
  if( a->node >= 0 ) {
    int cpu = node_cpu( a->node );
    if( cpu >= 0 ) { cpu_set_t s1; CPU_ZERO( &s1 ); CPU_SET( cpu, &s1 ); (void)pthread_setaffinity_np( pthread_self(), sizeof(s1), &s1 ); }
    link_bind( part, part_sz, a->node );
    link_bind( l->line[q], mc_bytes( a->depth ), a->node );
  }
  mc_init_lines( l->line[q], a->depth, 0UL );
  ulong c = h->part_off[q] / FDGPU_CHUNK_SZ;
  for( ulong p=q; p<a->n_payload; p+=Q ) {
    fdgpu_txnm_t * txnm = (fdgpu_txnm_t *)( l->dcache + c * FDGPU_CHUNK_SZ );
    memset( txnm, 0, FDGPU_TXNM_HDR_SZ );
    txnm->payload_sz = a->sz[p];
    memcpy( (uchar *)txnm + FDGPU_TXNM_HDR_SZ, a->payload + a->off[p], a->sz[p] );
    l->chunk[p] = (unsigned)c; l->psz[p] = a->sz[p];
    l->psig[p] = a->sz[p] ? a->payload[ a->off[p] ] : (uchar)0;
    c = fdgpu_dcache_compact_next( c, FDGPU_TXNM_HDR_SZ + a->sz[p], 0UL, ~0UL );
  }
  for( uchar * t = part + ( ( c * FDGPU_CHUNK_SZ - h->part_off[q] + 4095UL ) & ~4095UL ); t < part + part_sz; t += 4096 ) *t = 0;
  h->dc_node[q] = link_node_of( part );
  h->mc_node[q] = link_node_of( l->line[q] );
  return NULL;
}

/* where the link's memory is: each producer's dcache part and mcache NUMA node (q < producers), and of the link
   region as this process maps it, the bytes in 2 MiB pages (AnonHugePages / ShmemPmdMapped / FilePmdMapped, and
   Shared_/Private_Hugetlb for a link file on hugetlbfs, of its mapping in /proc/self/smaps) and its size; returns
   the producer count */
int
fdgpu_link_placement( fdgpu_link_t const * l, int * dc_node, int * mc_node, unsigned long * huge_bytes,
                      unsigned long * map_bytes ) {
  link_hdr_t const * h = l->h;
  for( int q=0; q<h->cfg.producers; q++ ) { dc_node[q] = h->dc_node[q]; mc_node[q] = h->mc_node[q]; }
  *huge_bytes = 0UL; *map_bytes = 0UL;
  FILE * f = fopen( "/proc/self/smaps", "r" );
  if( f ) {
    char line[ 512 ]; int in = 0;
    while( fgets( line, sizeof(line), f ) ) {
      ulong a, b;
      char * sp = strchr( line, ' ' ), * da = strchr( line, '-' );
      if( sp && da && da < sp && sscanf( line, "%lx-%lx ", &a, &b ) == 2 ) {   /* a mapping's header: "start-end perms ..." */
        in = (ulong)l->dcache >= a && (ulong)l->dcache < b;
        if( in ) *map_bytes += b - a;
        continue;
      }
      ulong kb;
      if( in && ( sscanf( line, "AnonHugePages: %lu kB", &kb ) == 1 || sscanf( line, "ShmemPmdMapped: %lu kB", &kb ) == 1 ||
                  sscanf( line, "FilePmdMapped: %lu kB", &kb ) == 1 || sscanf( line, "Shared_Hugetlb: %lu kB", &kb ) == 1 ||
                  sscanf( line, "Private_Hugetlb: %lu kB", &kb ) == 1 ) ) *huge_bytes += kb << 10;
    }
    fclose( f );
  }
  return h->cfg.producers;
}

fdgpu_link_t *
fdgpu_link_new( char const * path, fdgpu_stream_cfg_t const * cfg, uchar const * payload, unsigned const * off,
                unsigned short const * sz, ulong n_payload, ulong mcache_depth ) {
  if( !cfg || cfg->tiles < 1 || cfg->tiles > LINK_TILE_MAX || cfg->gpus < 1 || cfg->gpus > cfg->tiles || !n_payload ||
      !cfg->n_frags || !cfg->batch_txn || mcache_depth < 64 || cfg->producers < 0 || cfg->producers > LINK_PROD_MAX )
    return NULL;
  ulong Q = cfg->producers ? (ulong)cfg->producers : 1UL;
  ulong depth = pow2_up( mcache_depth );
  /* the in dcache in Q parts: producer q's payloads (p % Q == q: producer q's frag s is payload (s Q + q) %
     n_payload) in part q, each part 2 MiB aligned, so that each can live on its producer's NUMA node as the
     reference places each QUIC tile's out link in a workspace on that tile's node (src/disco/topo/fd_topob.c:
     505-540, fd_topo.c:82) */
  ulong part_off[ LINK_PROD_MAX + 1 ] = { 0 };
  for( ulong p=0; p<n_payload; p++ ) if( sz[p] > 1232U ) return NULL;
  for( ulong q=0; q<Q; q++ ) {
    ulong b = 0UL;
    for( ulong p=q; p<n_payload; p+=Q ) b += ( ( FDGPU_TXNM_HDR_SZ + sz[p] + 127UL ) >> 7 ) << 7;
    part_off[q+1] = ( ( part_off[q] + b ) + ( 2UL << 20 ) - 1UL ) & ~( ( 2UL << 20 ) - 1UL );
  }
  ulong in_bytes = part_off[Q];
  ulong T = (ulong)cfg->tiles;
  ulong o = al64( sizeof(link_hdr_t) );
  ulong off_mcache[ LINK_PROD_MAX ] = { 0 };
  o = ( o + 4095UL ) & ~4095UL;                /* page-aligned line arrays: registered with the GPU (overrun check) */
  for( ulong q=0; q<Q; q++ ) { off_mcache[q] = o;  o += mc_bytes( depth ); }
  ulong off_chunk  = o;  o = al64( o + n_payload * sizeof(unsigned) );
  ulong off_sz     = o;  o = al64( o + n_payload * sizeof(unsigned short) );
  ulong off_psig   = o;  o = al64( o + n_payload );
  ulong off_res    = o;  o = al64( o + T * sizeof(link_res_t) );
  ulong off_hist   = o;  o = al64( o + T * LH_N * sizeof(ulong) );
  ulong off_trace  = o;  o = al64( o + T * cfg->trace_cap * sizeof(fdgpu_link_trace_t) );
  o = ( o + ( 2UL << 20 ) - 1UL ) & ~( ( 2UL << 20 ) - 1UL );   /* (the parts' 2 MiB alignment holds in the region) */
  ulong off_dcache = o;  o += in_bytes + 4096UL;
  ulong total = ( o + 4095UL ) & ~4095UL;
  uchar * base;
  int shared = path != NULL;
  if( shared ) {
    int fd = open( path, O_RDWR | O_CREAT | O_EXCL, 0600 );
    if( fd < 0 ) return NULL;
    /* a path on hugetlbfs (the reference's workspaces: fd_shmem's .huge / .gigantic mounts) gives the link huge
       pages whatever shmem_enabled says: the file's size is then a whole number of its pages */
    struct statfs sfs;
    if( !fstatfs( fd, &sfs ) && (ulong)sfs.f_type == 0x958458f6UL && sfs.f_bsize > 0 )
      total = ( total + (ulong)sfs.f_bsize - 1UL ) / (ulong)sfs.f_bsize * (ulong)sfs.f_bsize;
    if( ftruncate( fd, (off_t)total ) ) { close( fd ); unlink( path ); return NULL; }
    base = (uchar *)mmap( NULL, total, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0 );
    close( fd );
    if( base == MAP_FAILED ) { unlink( path ); return NULL; }
  }
  uchar * map = base; ulong map_sz = total;
  if( !shared ) {
    /* The reference's links live in workspaces of huge (2 MiB) or gigantic pages (fd_wksp); the GPU reads
       this region frag by frag over PCIe (zero-copy intake), and with 4 KiB pages every frag is a GPU TLB
       miss in a 1+ GB region.  Transparent huge pages where the kernel allows them (madvise mode): a 2 MiB
       aligned region advised before first touch (cfg.no_huge_pages: 4 KiB pages, A/B). */
    ulong const huge = 2UL << 20;
    map_sz = total + ( cfg->no_huge_pages ? 0UL : huge );
    map = (uchar *)mmap( NULL, map_sz, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0 );
    if( map == MAP_FAILED ) return NULL;
    base = map;
    if( !cfg->no_huge_pages ) {
      base = (uchar *)( ( (ulong)map + huge - 1UL ) & ~( huge - 1UL ) );
      (void)madvise( base, total, MADV_HUGEPAGE );   /* whole 2 MiB extents in it become huge pages */
    }
  } else if( !cfg->no_huge_pages ) {
    (void)madvise( base, total, MADV_HUGEPAGE );    /* shmem: honoured only where shmem_enabled allows it */
  }
  fdgpu_link_t * l = (fdgpu_link_t *)calloc( 1, sizeof(fdgpu_link_t) );
  if( !l ) { munmap( map, map_sz ); return NULL; }
  l->base = base; l->sz = total; l->map = map; l->map_sz = map_sz; l->shared = shared; l->h = (link_hdr_t *)base;
  if( shared ) snprintf( l->path, sizeof(l->path), "%s", path );
  link_hdr_t * h = l->h;
  memset( (void *)h, 0, sizeof(link_hdr_t) );
  h->total_sz = total; h->cfg = *cfg; h->cfg.producers = (int)Q;
  h->depth = depth; h->n_payload = n_payload; h->in_bytes = in_bytes;
  for( ulong q=0; q<Q; q++ ) h->off_mcache[q] = off_mcache[q];
  h->off_dcache = off_dcache; h->off_chunk = off_chunk; h->off_sz = off_sz; h->off_psig = off_psig;
  h->off_res = off_res; h->off_hist = off_hist; h->off_trace = off_trace;
  for( ulong q=0; q<=Q; q++ ) h->part_off[q] = part_off[q];
  link_view( l );
  memset( (void *)l->res, 0, T * sizeof(link_res_t) );
  memset( (void *)l->hist, 0, T * LH_N * sizeof(ulong) );
  /* each producer's mcache and dcache part first touched by a thread on its node (cfg.prod_node; the memory
     policy bound there too where the kernel allows it), its payloads prefilled (what QUIC reassembly leaves) */
  link_fill_arg_t fa[ LINK_PROD_MAX ];
  pthread_t fth[ LINK_PROD_MAX ];
  for( ulong q=0; q<Q; q++ ) {
    fa[q].l = l; fa[q].q = (int)q; fa[q].Q = (int)Q; fa[q].node = cfg->prod_node[q] - 1; fa[q].depth = depth;
    fa[q].payload = payload; fa[q].off = off; fa[q].sz = sz; fa[q].n_payload = n_payload;
    if( pthread_create( &fth[q], NULL, link_fill, &fa[q] ) ) link_fill( &fa[q] ), fth[q] = 0;
  }
  for( ulong q=0; q<Q; q++ ) if( fth[q] ) pthread_join( fth[q], NULL );
  atomic_store_explicit( &h->joined, 1UL, memory_order_relaxed );
  atomic_store_explicit( &h->magic, LINK_MAGIC, memory_order_release );
  return l;
}

fdgpu_link_t *
fdgpu_link_join( char const * path, double timeout_s ) {
  ulong t0 = now_ns(), lim = (ulong)( timeout_s * 1e9 );
  int fd = -1;
  for(;;) {                                    /* the creator may not have made the file yet */
    fd = open( path, O_RDWR );
    if( fd >= 0 ) {
      struct stat st;
      if( !fstat( fd, &st ) && (ulong)st.st_size >= sizeof(link_hdr_t) ) {
        /* (whole pages of the file's own size: a link on hugetlbfs is mapped and unmapped in huge pages) */
        ulong pg = st.st_blksize > 4096 ? (ulong)st.st_blksize : 4096UL;
        ulong hl = ( sizeof(link_hdr_t) + pg - 1UL ) / pg * pg;
        link_hdr_t * h = (link_hdr_t *)mmap( NULL, hl, PROT_READ, MAP_SHARED, fd, 0 );
        if( h != MAP_FAILED ) {
          int ok = atomic_load_explicit( &h->magic, memory_order_acquire ) == LINK_MAGIC;
          ulong total = h->total_sz;
          munmap( (void *)h, hl );
          if( ok && (ulong)st.st_size >= total ) {
            /* every page mapped now (MAP_POPULATE): a tile that joins reads records all over the in dcache, and
               would otherwise take a page fault per page at the start of its stream (measured: multi-ms stalls
               of a served tile process at 10M frags/s) */
            uchar * base = (uchar *)mmap( NULL, total, PROT_READ | PROT_WRITE, MAP_SHARED | MAP_POPULATE, fd, 0 );
            close( fd );
            if( base == MAP_FAILED ) return NULL;
            fdgpu_link_t * l = (fdgpu_link_t *)calloc( 1, sizeof(fdgpu_link_t) );
            if( !l ) { munmap( base, total ); return NULL; }
            snprintf( l->path, sizeof(l->path), "%s", path );
            l->base = base; l->sz = total; l->map = base; l->map_sz = total; l->shared = 1; l->h = (link_hdr_t *)base;
            link_view( l );
            atomic_fetch_add( &l->h->joined, 1UL );
            return l;
          }
        }
      }
      close( fd );
    }
    if( now_ns() - t0 > lim ) return NULL;
    usleep( 2000 );
  }
}

void
fdgpu_link_delete( fdgpu_link_t * l ) {
  if( !l ) return;
  if( l->registered ) {
    fdgpu_host_unregister( l->dcache );
    for( int q=0; q<l->h->cfg.producers; q++ ) fdgpu_host_unregister( l->line[q] );
  }
  munmap( l->map, l->map_sz );
  if( l->trace_own ) for( int i=0; i<LINK_TILE_MAX; i++ ) free( l->trace[i] );
  free( l );
}

int
fdgpu_link_set_trace( fdgpu_link_t * l, ulong cap ) {
  if( l->h->cfg.trace_cap ) return cap == l->h->cfg.trace_cap ? 0 : -1;   /* the link's own traces (cfg.trace_cap) */
  for( int i=0; i<LINK_TILE_MAX; i++ ) {
    if( l->trace_own ) free( l->trace[i] );
    l->trace[i] = NULL;
  }
  for( int i=0; i<l->h->cfg.tiles && i<LINK_TILE_MAX; i++ ) l->res[i].trace_cnt = 0UL;
  l->trace_cap = 0UL; l->trace_own = 1;
  if( !cap ) return 0;
  for( int i=0; i<l->h->cfg.tiles && i<LINK_TILE_MAX; i++ )
    if( !( l->trace[i] = (fdgpu_link_trace_t *)calloc( cap, sizeof(fdgpu_link_trace_t) ) ) ) return -1;
  l->trace_cap = cap;
  return 0;
}

ulong
fdgpu_link_trace( fdgpu_link_t const * l, int tile, fdgpu_link_trace_t * out, ulong max ) {
  if( tile < 0 || tile >= LINK_TILE_MAX || !l->trace[tile] ) return 0UL;
  ulong c = l->res[tile].trace_cnt, n = c < max ? c : max;
  memcpy( out, l->trace[tile], n * sizeof(fdgpu_link_trace_t) );
  return n;
}

/* the verdicts a tile just returned, in order (fdgpu_link_set_trace): a published frag's record is
   hashed where the tile published it, in its out dcache, with the alignment byte between an odd-sized
   payload and the fd_txn_t taken as 0 (the reference leaves whatever the chunk held there) */
static void
link_trace( fdgpu_link_t * l, int idx, fdgpu_vtile_t * vt, fdgpu_vtile_done_t const * d, ulong n ) {
  fdgpu_link_trace_t * t = l->trace[idx];
  if( !t ) return;
  uchar const * out = fdgpu_vtile_out_dcache( vt );
  for( ulong i=0; i<n && l->res[idx].trace_cnt < l->trace_cap; i++ ) {
    fdgpu_link_trace_t * e = &t[ l->res[idx].trace_cnt++ ];
    e->seq = d[i].seq; e->in_idx = d[i].in_idx; e->tag = d[i].tag; e->result = d[i].result; e->rec_sz = (unsigned)d[i].sz;
    e->rec_hash = 0UL;
    if( d[i].result == FDGPU_VTILE_PUBLISH && d[i].sz <= VT_RESERVE_MAX ) {
      uchar rec[ VT_RESERVE_MAX ];
      memcpy( rec, out + d[i].chunk * FDGPU_CHUNK_SZ, d[i].sz );
      ulong pe = FDGPU_TXNM_HDR_SZ + ((fdgpu_txnm_t const *)rec)->payload_sz;
      if( ( pe & 1UL ) && pe < d[i].sz ) rec[ pe ] = 0;
      e->rec_hash = fdgpu_xxh64( 0UL, rec, d[i].sz );
    }
  }
}

ulong fdgpu_link_joined( fdgpu_link_t const * l ) { return atomic_load( &l->h->joined ); }
fdgpu_mcache_t * fdgpu_link_mcache( fdgpu_link_t * l ) { return &l->mc[0]; }
unsigned char *  fdgpu_link_dcache( fdgpu_link_t * l ) { return l->dcache; }

/* the reference's verify-tile -> GPU binding: tile i drives GPU i % G and
   runs in that GPU's process; the tiles of process proc, ascending */
int
fdgpu_link_tiles_of( int tiles, int gpus, int proc, int * out ) {
  int n = 0;
  if( tiles < 1 || gpus < 1 || proc < 0 || proc >= gpus ) return 0;
  for( int i=0; i<tiles; i++ ) if( i % gpus == proc ) out[n++] = i;
  return n;
}
void  fdgpu_link_cfg( fdgpu_link_t const * l, fdgpu_stream_cfg_t * cfg ) { *cfg = l->h->cfg; }

typedef struct { fdgpu_link_t * l; int q, cpu; } link_prod_arg_t;

static void link_pin( int cpu );

/* The calling thread's CPU time and involuntary context switches: on a shared host a pinned
   thread that loses its core to another process shows CPU time below its wall time. */
static void thread_usage( ulong * cpu_ns, ulong * nivcsw ) {
  struct timespec ts; struct rusage ru;
  *cpu_ns = clock_gettime( CLOCK_THREAD_CPUTIME_ID, &ts ) ? 0UL : (ulong)ts.tv_sec * 1000000000UL + (ulong)ts.tv_nsec;
  *nivcsw = getrusage( RUSAGE_THREAD, &ru ) ? 0UL : (ulong)ru.ru_nivcsw;
}

/* producer q (one of the reference's QUIC tiles): publishes its frags on its
   own mcache, seq 0 .. n_q-1, frag s pointing at payload (s Q + q) % n_payload */
static void * link_producer( void * _a ) {
  link_prod_arg_t * a = (link_prod_arg_t *)_a;
  link_pin( a->cpu );
  fdgpu_link_t * l = a->l;
  link_hdr_t * h = l->h;
  h->prod_cpu[ a->q ] = a->cpu;
  fdgpu_stream_cfg_t const * c = &h->cfg;
  ulong const q = (ulong)a->q, Q = (ulong)c->producers;
  ulong T = (ulong)c->tiles, mask = h->depth - 1UL, n_q = prod_frags( c->n_frags, Q, q );
  ulong t_wait0 = now_ns();
  if( q == 0UL ) {
    while( atomic_load( &h->tiles_ready ) < T ) {   /* every tile has its GPU context */
      if( atomic_load( &h->fail ) ) return NULL;
      if( now_ns() - t_wait0 > 120000000000UL ) {
        fprintf( stderr, "fdgpu_link: producer waited 120 s for %lu tiles (%lu ready)\n", T, atomic_load( &h->tiles_ready ) );
        atomic_store( &h->fail, 6 ); return NULL;
      }
    }
    h->t_start = now_ns();
    atomic_store_explicit( &h->go, 1UL, memory_order_release );
  } else {
    while( !atomic_load_explicit( &h->go, memory_order_acquire ) ) {
      if( atomic_load( &h->fail ) ) return NULL;
      if( now_ns() - t_wait0 > 180000000000UL ) { atomic_store( &h->fail, 6 ); return NULL; }
    }
  }
  ulong t0 = now_ns(), cpu0, iv0;
  thread_usage( &cpu0, &iv0 );
  double rate = c->rate_fps > 0. ? c->rate_fps / (double)Q : 0.;   /* the offered load, split over the producers */
  mc_line_t * line = l->line[q];
  ulong cr_until = 0UL, wait_ns = 0UL;      /* may publish seq < cr_until */
  for( ulong seq=0; seq<n_q; seq++ ) {
    if( c->reliable ) {
      ulong t_wait = 0UL;
      if( seq >= cr_until ) t_wait = now_ns();
      while( seq >= cr_until ) {
        if( atomic_load_explicit( &h->fail, memory_order_relaxed ) ) return NULL;
        if( now_ns() - t_wait > 30000000000UL ) {                  /* watchdog: 30 s without credits */
          fprintf( stderr, "fdgpu_link: producer %lu starved of credits at seq %lu\n", q, seq );
          atomic_store( &h->fail, 4 ); return NULL;
        }
        ulong lo = ~0UL;
        for( ulong t=0; t<T; t++ ) { ulong f = atomic_load_explicit( &h->fseq[q][t].v, memory_order_acquire ); if( f < lo ) lo = f; }
        cr_until = lo + h->depth/2;
      }
      if( t_wait ) wait_ns += now_ns() - t_wait;
    }
    if( rate > 0. ) {
      ulong due = t0 + (ulong)( (double)seq * 1e9 / rate );
      while( now_ns() < due ) ;
    }
    ulong p = ( seq * Q + q ) % h->n_payload;
    unsigned ts = (unsigned)now_ns();
    mc_publish( &line[ seq & mask ], seq, 0UL, l->chunk[p], (unsigned)( FDGPU_TXNM_HDR_SZ + l->psz[p] ), ts, ts );
  }
  h->prod_wait_ns[q] = wait_ns;
  h->prod_end[q] = now_ns();
  ulong cpu1, iv1;
  thread_usage( &cpu1, &iv1 );
  h->prod_cpu_ns[q] = cpu1 - cpu0; h->prod_wall_ns[q] = h->prod_end[q] - t0; h->prod_nivcsw[q] = iv1 - iv0;
  return NULL;
}

/* CPU placement of the link's threads.  The reference pins every tile to
   a core of its own (the [layout] affinity); here, by default, the
   producer and this process's tiles take one hardware thread each of
   distinct physical cores, on the GPU's NUMA node, filling one L3 (CCD)
   before the next -- the mcache lines the producer writes and every tile
   polls then move between cores that share an L3.  Process proc starts
   at the L3 group proc % groups, so the processes of a multi-GPU run do
   not share cores.  Cores another process kept busy over a 30 ms sample
   are passed over while enough idle ones remain (a shared host).  Env
   FDGPU_LINK_PIN: 0 = no pinning, "lowest" = no sample, an explicit comma
   list of CPUs (producer first, then the tiles), else automatic. */
#define LINK_CPU_MAX 1024
static int cpulist_read( char const * path, uchar * set ) {
  FILE * f = fopen( path, "r" );
  if( !f ) return -1;
  char buf[ 4096 ]; size_t n = fread( buf, 1, sizeof(buf)-1, f ); fclose( f ); buf[n] = 0;
  char * c = buf;
  while( *c ) {
    char * e; long a = strtol( c, &e, 10 ), b = a;
    if( e == c ) break;
    if( *e == '-' ) { c = e + 1; b = strtol( c, &e, 10 ); }
    for( long i=a; i<=b && i<LINK_CPU_MAX; i++ ) if( i >= 0 ) set[i] = 1;
    c = e; if( *c == ',' ) c++; else break;
  }
  return 0;
}
static int cpu_first_of( char const * fmt, int cpu ) {          /* lowest CPU of a sysfs cpulist */
  char path[ 160 ]; snprintf( path, sizeof(path), fmt, cpu );
  static __thread uchar set[ LINK_CPU_MAX ];
  memset( set, 0, sizeof(set) );
  if( cpulist_read( path, set ) ) return cpu;
  for( int i=0; i<LINK_CPU_MAX; i++ ) if( set[i] ) return i;
  return cpu;
}
/* Busy fraction of each CPU over `ms` milliseconds (/proc/stat): the cores another process keeps busy
   are not worth pinning a spinning tile to.  Returns 0 on success. */
static int cpu_busy_sample( double * busy, int ms ) {
  ulong t0[ LINK_CPU_MAX ] = { 0 }, i0[ LINK_CPU_MAX ] = { 0 };   /* (on the stack: link_run may run in several threads) */
  for( int pass=0; pass<2; pass++ ) {
    FILE * f = fopen( "/proc/stat", "r" );
    if( !f ) return -1;
    char line[ 512 ];
    while( fgets( line, sizeof(line), f ) ) {
      int cpu; ulong v[8] = { 0 };
      if( strncmp( line, "cpu", 3 ) || line[3] < '0' || line[3] > '9' ) continue;
      if( sscanf( line + 3, "%d %lu %lu %lu %lu %lu %lu %lu %lu", &cpu, v, v+1, v+2, v+3, v+4, v+5, v+6, v+7 ) < 5 ) continue;
      if( cpu < 0 || cpu >= LINK_CPU_MAX ) continue;
      ulong tot = 0UL; for( int k=0; k<8; k++ ) tot += v[k];
      ulong idle = v[3] + v[4];                                  /* idle + iowait */
      if( !pass ) { t0[cpu] = tot; i0[cpu] = idle; }
      else {
        ulong dt = tot - t0[cpu], di = idle - i0[cpu];
        busy[cpu] = dt ? 1. - (double)di / (double)dt : 0.;
      }
    }
    fclose( f );
    if( !pass ) usleep( (useconds_t)ms * 1000U );
  }
  return 0;
}

/* HIP device -> NUMA node from sysfs alone (fdgpu_gpu_numa_node_sysfs, include/fd_verify_gpu.h).  HIP
   numbers the GPU agents of the KFD topology (nodes with SIMDs) in node order, after ROCR_VISIBLE_DEVICES
   (indices into all of them) and then HIP_VISIBLE_DEVICES / CUDA_VISIBLE_DEVICES (indices into what ROCr
   shows).  A node's location_id is its PCI bus << 8 | devfn and `domain` its PCI domain. */
static int visible_pick( char const * env, int * ids, int n ) {   /* ids[0..n) filtered by a comma list of indices */
  if( !env || !*env ) return n;
  int out[ 64 ], m = 0;
  char const * c = env;
  while( *c && m < 64 ) {
    char * e; long v = strtol( c, &e, 10 );
    if( e == c ) return -1;                                       /* (UUIDs: not resolved here) */
    if( v >= 0 && v < n ) out[m++] = ids[v];
    c = *e == ',' ? e + 1 : e;
    if( *e && *e != ',' ) return -1;
  }
  for( int i=0; i<m; i++ ) ids[i] = out[i];
  return m;
}

static long sysfs_prop( char const * path, char const * key ) {
  FILE * f = fopen( path, "r" );
  if( !f ) return -1L;
  char line[ 256 ]; long v = -1L; size_t kl = strlen( key );
  while( fgets( line, sizeof(line), f ) )
    if( !strncmp( line, key, kl ) && line[kl] == ' ' ) { v = strtol( line + kl + 1, NULL, 10 ); break; }
  fclose( f );
  return v;
}

int
fdgpu_gpu_numa_node_sysfs( char const * root, int device ) {
  if( !root ) root = "/sys";
  if( device < 0 ) return -1;
  char path[ 512 ];
  snprintf( path, sizeof(path), "%s/class/kfd/kfd/topology/nodes", root );
  DIR * d = opendir( path );
  if( !d ) return -1;
  int nodes[ 64 ], nn = 0;
  struct dirent * e;
  while( ( e = readdir( d ) ) && nn < 64 ) {
    char * end; long v = strtol( e->d_name, &end, 10 );
    if( end == e->d_name || *end ) continue;
    nodes[nn++] = (int)v;
  }
  closedir( d );
  for( int i=1; i<nn; i++ ) for( int j=i; j>0 && nodes[j-1] > nodes[j]; j-- ) { int t = nodes[j]; nodes[j] = nodes[j-1]; nodes[j-1] = t; }
  int gpus[ 64 ], ng = 0;
  for( int i=0; i<nn; i++ ) {
    snprintf( path, sizeof(path), "%s/class/kfd/kfd/topology/nodes/%d/properties", root, nodes[i] );
    if( sysfs_prop( path, "simd_count" ) > 0 ) gpus[ng++] = nodes[i];
  }
  ng = visible_pick( getenv( "ROCR_VISIBLE_DEVICES" ), gpus, ng );
  char const * hv = getenv( "HIP_VISIBLE_DEVICES" );
  if( !hv || !*hv ) hv = getenv( "CUDA_VISIBLE_DEVICES" );
  if( ng > 0 ) ng = visible_pick( hv, gpus, ng );
  if( ng <= 0 || device >= ng ) return -1;
  snprintf( path, sizeof(path), "%s/class/kfd/kfd/topology/nodes/%d/properties", root, gpus[device] );
  long loc = sysfs_prop( path, "location_id" ), dom = sysfs_prop( path, "domain" );
  if( loc < 0 ) return -1;
  if( dom < 0 ) dom = 0;
  snprintf( path, sizeof(path), "%s/bus/pci/devices/%04lx:%02lx:%02lx.%lx/numa_node", root, (ulong)dom,
            ( (ulong)loc >> 8 ) & 0xffUL, ( (ulong)loc >> 3 ) & 0x1fUL, (ulong)loc & 7UL );
  FILE * f = fopen( path, "r" );
  if( !f ) return -1;
  int node = -1;
  if( fscanf( f, "%d", &node ) != 1 ) node = -1;
  fclose( f );
  return node;
}

/* n CPUs for this process's link threads, in the order producers, tiles, launch threads, copy threads:
   one hardware thread per core, on the GPU's NUMA node when it has them, idle cores first, filling one L3
   group (a CCD) after another from group proc (so processes spread).  n_pair: the producers plus tiles --
   a frag's mcache line and record header move from the producer's core to a tile's, a coherence miss per
   frag that costs about twice as much across L3 groups -- so the first group taken is the first, from
   proc's, with n_pair idle cores, when there is one. */
static int
link_pick_cpus( int device, int proc, int n, int n_pair, int * out, int gpu_calls ) {
  char const * env = getenv( "FDGPU_LINK_PIN" );
  if( env && !strcmp( env, "0" ) ) return 0;
  int got = 0;
  if( env && *env >= '0' && *env <= '9' ) {                      /* explicit list (anything else: automatic) */
    char const * c = env;
    while( *c && got < n ) { char * e; long v = strtol( c, &e, 10 ); if( e == c ) break; out[got++] = (int)v; c = *e ? e + 1 : e; }
    return got;
  }
  cpu_set_t aff; CPU_ZERO( &aff );
  if( sched_getaffinity( 0, sizeof(aff), &aff ) ) return 0;
  uchar node_set[ LINK_CPU_MAX ];
  memset( node_set, 0, sizeof(node_set) );
  /* the device's node: from its bus id (a GPU call), or from sysfs alone in a process that must not touch the
     GPU before it forks its tiles (served tiles) */
  int node = gpu_calls ? fdgpu_device_numa_node( device ) : fdgpu_gpu_numa_node_sysfs( NULL, device ), use_node = 0;
  if( node >= 0 ) {
    char path[ 96 ]; snprintf( path, sizeof(path), "/sys/devices/system/node/node%d/cpulist", node );
    use_node = !cpulist_read( path, node_set );
  }
  /* a shared machine: skip cores (either hardware thread) that another process kept busy over a short
     sample, unless too few idle ones are left (FDGPU_LINK_PIN=lowest: no sample, the lowest cores) */
  double busy[ LINK_CPU_MAX ];
  memset( busy, 0, sizeof(busy) );
  if( !( env && !strcmp( env, "lowest" ) ) ) cpu_busy_sample( busy, 30 );
  /* candidate cores: one hardware thread (the lowest sibling) of each allowed core */
  int cand[ LINK_CPU_MAX ], grp[ LINK_CPU_MAX ], nc = 0;
  uchar hot[ LINK_CPU_MAX ];
  uchar sib[ LINK_CPU_MAX ];
  for( int pass=0; pass<2 && !nc; pass++ )                       /* pass 1: ignore the node if it has no allowed CPU */
    for( int c=0; c<LINK_CPU_MAX && c<CPU_SETSIZE; c++ ) {
      if( !CPU_ISSET( c, &aff ) || ( pass==0 && use_node && !node_set[c] ) ) continue;
      if( cpu_first_of( "/sys/devices/system/cpu/cpu%d/topology/thread_siblings_list", c ) != c ) continue;
      char path[ 160 ];
      snprintf( path, sizeof(path), "/sys/devices/system/cpu/cpu%d/topology/thread_siblings_list", c );
      memset( sib, 0, sizeof(sib) ); sib[c] = 1;
      cpulist_read( path, sib );
      double b = 0.;
      for( int k=0; k<LINK_CPU_MAX; k++ ) if( sib[k] && busy[k] > b ) b = busy[k];
      hot[nc] = b > 0.25;
      cand[nc] = c; grp[nc] = cpu_first_of( "/sys/devices/system/cpu/cpu%d/cache/index3/shared_cpu_list", c ); nc++;
    }
  if( !nc ) return 0;
  int gid[ LINK_CPU_MAX ], ng = 0;                               /* L3 groups in CPU order */
  for( int i=0; i<nc; i++ ) { int k=0; while( k<ng && gid[k] != grp[i] ) k++; if( k==ng ) gid[ng++] = grp[i]; }
  int r0 = 0;                                                    /* the first group with room for the pairs */
  for( int r=0; r<ng; r++ ) {
    int g = gid[ ( proc + r ) % ng ], idle = 0;
    for( int i=0; i<nc; i++ ) idle += grp[i] == g && !hot[i];
    if( idle >= n_pair ) { r0 = r; break; }
  }
  for( int pass=0; pass<2 && got<n; pass++ )                    /* pass 0: idle cores only, then the rest */
    for( int r=0; r<ng && got<n; r++ ) {
      int g = gid[ ( proc + r0 + r ) % ng ];
      for( int i=0; i<nc && got<n; i++ ) {
        if( grp[i] != g || ( pass==0 && hot[i] ) ) continue;
        int dup = 0; for( int k=0; k<got; k++ ) dup |= out[k] == cand[i];
        if( !dup ) out[got++] = cand[i];
      }
    }
  return got;
}
/* producers placed on a node other than the GPU's (cfg.prod_node: e.g. the cross-socket arm) run on that node:
   cpus[i] of producer i becomes an allowed CPU of that node (one hardware thread per core) not otherwise taken */
static void link_place_producers( fdgpu_stream_cfg_t const * c, int const * myq, int np, int * cpus, int ncpu, int gpu_node ) {
  for( int i=0; i<np && i<ncpu; i++ ) {
    int node = c->prod_node[ myq[i] ] - 1;
    if( node < 0 || node == gpu_node ) continue;
    char path[ 96 ]; snprintf( path, sizeof(path), "/sys/devices/system/node/node%d/cpulist", node );
    uchar set[ LINK_CPU_MAX ]; memset( set, 0, sizeof(set) );
    if( cpulist_read( path, set ) ) continue;
    cpu_set_t aff; CPU_ZERO( &aff );
    if( sched_getaffinity( 0, sizeof(aff), &aff ) ) continue;
    for( int k=0; k<LINK_CPU_MAX && k<CPU_SETSIZE; k++ ) {
      if( !set[k] || !CPU_ISSET( k, &aff ) ) continue;
      if( cpu_first_of( "/sys/devices/system/cpu/cpu%d/topology/thread_siblings_list", k ) != k ) continue;
      int used = 0; for( int j=0; j<ncpu; j++ ) used |= cpus[j] == k;
      if( !used ) { cpus[i] = k; break; }
    }
  }
}

static void link_pin( int cpu ) {
  if( cpu < 0 ) return;
  cpu_set_t s; CPU_ZERO( &s ); CPU_SET( cpu, &s );
  if( pthread_setaffinity_np( pthread_self(), sizeof(s), &s ) )
    fprintf( stderr, "fdgpu_link: could not pin to CPU %d\n", cpu );
}

typedef struct {
  fdgpu_link_t * l; int idx, device, cpu, lcpu, ccpu[ FDGPU_VTILE_COPY_THREADS_MAX ];
  fdgpu_vsvc_t * svc; int client;                /* served tiles (cfg.svc): the service and this tile's client slot */
} link_tile_arg_t;
/* lcpu: its launch thread's CPU, ccpu: its copy threads' */

/* per-link state of a tile */
typedef struct {
  ulong seq;                     /* next seq of the link this tile has not consumed (own or not) */
  ulong n;                       /* frags the link's producer publishes */
  ulong credited;                /* last credit returned */
  ulong app, fin;                /* own frags handed to during_frag / returned by after_frags */
} link_in_t;

/* credit a tile returns to producer q: every seq below it may be
   overwritten.  With zero-copy intake a frag's bytes must survive until
   the GPU has copied them (the stem's during_frag copy, done by the GPU:
   fdgpu_vtile_copy_state), so while frags of the link are not yet copied
   the credit stops at the first seq after the link's last copied frag
   (copies complete in seq order per link, so that is at or below the
   oldest uncopied one).  The verdict does not hold the link. */
static void link_credit( link_hdr_t * h, int q, int idx, link_in_t const * in, fdgpu_vtile_t const * vt ) {
  ulong c = in->seq;
  if( h->cfg.zero_copy ) { ulong cn; if( fdgpu_vtile_copy_state( vt, q, &cn ) && cn < c ) c = cn; }
  atomic_store_explicit( &h->fseq[q][idx].v, c, memory_order_release );
}

/* own frags (q % T == idx) in [a, b) */
static ulong own_in( ulong a, ulong b, ulong T, ulong idx ) {
  if( b <= a ) return 0UL;
  ulong ca = a > idx ? ( a - idx + T - 1UL ) / T : 0UL;   /* #own q < a */
  ulong cb = b > idx ? ( b - idx + T - 1UL ) / T : 0UL;   /* #own q < b */
  return cb - ca;
}

ulong
fdgpu_link_anomalies( fdgpu_link_t const * l, int tile, fdgpu_link_anomaly_t * out, ulong max ) {
  if( tile < 0 || tile >= LINK_TILE_MAX ) return 0UL;
  if( tile >= l->h->cfg.tiles ) return 0UL;
  link_res_t const * r = &l->res[tile];
  ulong n = r->anom_cnt < LINK_ANOM_MAX ? r->anom_cnt : LINK_ANOM_MAX;
  if( n > max ) n = max;
  memcpy( out, r->anom, n * sizeof(fdgpu_link_anomaly_t) );
  return r->anom_cnt;
}

ulong
fdgpu_link_anomaly_results( fdgpu_link_t const * l, int tile, ulong * cnt ) {
  if( tile < 0 || tile >= LINK_TILE_MAX || tile >= l->h->cfg.tiles ) return 0UL;
  link_res_t const * r = &l->res[tile];
  memcpy( cnt, r->anom_by_result, sizeof(r->anom_by_result) );
  return r->anom_cnt;
}

static void
link_account( fdgpu_link_t * l, int idx, fdgpu_vtile_done_t const * d, ulong n, ulong * sigs, ulong * lh, ulong * lmax,
              ulong * t_last, link_in_t * in, uchar * pub ) {
  /* bench accounting only (not after_frag): the signature count comes from
     the link's per-payload table, not from the (cold) record in the out dcache.  pub: a bit per payload this
     tile has published -- the link's payloads recycle, so a dedup failure of a payload the tile published
     before is the tcache doing its job (its tag is still there: the tile lost or saw overrun most of the frags
     since), not an anomaly */
  ulong t = now_ns(), np = l->h->n_payload, Q = (ulong)l->h->cfg.producers;
  ulong pmask = ( np & ( np - 1UL ) ) ? 0UL : np - 1UL;   /* a power-of-two payload count: a mask, not a division */
  for( ulong i=0; i<n; i++ ) {
    ulong lat = t - d[i].tsorig;
    lh[ lh_idx( lat ) ]++;
    if( lat > *lmax ) *lmax = lat;
    int q = (int)d[i].in_idx;                      /* < Q: the tile handed it over with its link */
    ulong s = d[i].seq;
    in[q].fin++;
    ulong pi = pmask ? ( ( s * Q + (ulong)q ) & pmask ) : ( s * Q + (ulong)q ) % np;
    if( d[i].result == FDGPU_VTILE_PUBLISH || d[i].result == FDGPU_VTILE_VERIFY_FAIL || d[i].result == FDGPU_VTILE_DEDUP_FAIL )
      *sigs += l->psig[ pi ];
    if( d[i].result == FDGPU_VTILE_PUBLISH ) { if( pub ) pub[ pi >> 3 ] |= (uchar)( 1u << ( pi & 7UL ) ); continue; }
    if( d[i].result == FDGPU_VTILE_DEDUP_FAIL && pub && ( pub[ pi >> 3 ] >> ( pi & 7UL ) & 1 ) ) {
      l->res[idx].anom_by_result[ 0 ]++;           /* (slot 0, PUBLISH, never an anomaly: the recycled dedups) */
      continue;
    }
    if( __builtin_expect( d[i].result != FDGPU_VTILE_OVERRUN, 0 ) ) {
      ulong k = l->res[idx].anom_cnt++;
      l->res[idx].anom_by_result[ d[i].result & 7 ]++;
      if( k < LINK_ANOM_MAX ) {
        fdgpu_link_anomaly_t * e = &l->res[idx].anom[k];
        e->seq = s; e->in_idx = d[i].in_idx; e->tag = d[i].tag; e->result = d[i].result; e->code = d[i].code;
        e->payload_idx = pi;                         /* the link's layout: producer q's frag s */
        e->ctx = d[i].ctx; e->batch_txns = d[i].batch_txns; e->batch_pos = d[i].batch_pos; e->path = d[i].path;
      }
    }
  }
  if( n ) *t_last = t;
}

/* 1 if this process has the GPU open: a descriptor on /dev/kfd or a /dev/dri node (a HIP context's) */
static int proc_has_gpu_open( void ) {
  DIR * d = opendir( "/proc/self/fd" );
  if( !d ) return -1;
  int found = 0;
  struct dirent * e;
  while( ( e = readdir( d ) ) && !found ) {
    char p[ 320 ], t[ 256 ];
    snprintf( p, sizeof(p), "/proc/self/fd/%s", e->d_name );
    ssize_t n = readlink( p, t, sizeof(t) - 1 );
    if( n <= 0 ) continue;
    t[n] = 0;
    found = !strncmp( t, "/dev/kfd", 8 ) || !strncmp( t, "/dev/dri/", 9 );
  }
  closedir( d );
  return found;
}

static void * link_tile( void * _a ) {
  link_tile_arg_t * a = (link_tile_arg_t *)_a;
  link_pin( a->cpu );                          /* before any allocation: first touch on the tile's node */
  fdgpu_link_t * l = a->l;
  link_hdr_t * h = l->h;
  fdgpu_stream_cfg_t const * c = &h->cfg;
  int idx = a->idx;
  ulong const T = (ulong)c->tiles, mask = h->depth - 1UL, Q = (ulong)c->producers;
  /* out dcache: room for the frags a tile can have pending (its contexts' launched and filling
     batches), 6 batch limits' worth: with 3 a 2-tile max-rate run blocked in drains (16.7M vs
     18.8M sigs/s, profiles/r02/stream/sweep_depth.md) */
  ulong mult = c->out_mult ? c->out_mult : 6UL;
  fdgpu_vtile_opts_t vo;
  memset( &vo, 0, sizeof(vo) );
  vo.nctx = c->nctx; vo.copy_wait_ns = c->copy_wait_ns; vo.copy_min = c->copy_min; vo.gather_cus = c->gather_cus;
  vo.max_uncopied = c->max_uncopied; vo.cu_split = c->cu_split; vo.cu_exclusive = c->cu_exclusive;
  vo.launcher = c->launcher; vo.launcher_core = c->launcher && a->lcpu >= 0 ? a->lcpu + 1 : 0;
  vo.copy_threads = c->zero_copy ? c->copy_threads : 0;
  vo.min_batch = c->min_batch; vo.small_max = c->small_max; vo.lat_share = c->lat_share;
  for( int i=0; i<vo.copy_threads && i<FDGPU_VTILE_COPY_THREADS_MAX; i++ ) vo.copy_cores[i] = a->ccpu[i] >= 0 ? a->ccpu[i] + 1 : 0;
  fdgpu_vtile_t * vt = a->svc ? fdgpu_vtile_new_svc( a->svc, a->client, 1UL<<16, 0x5eedUL + (ulong)idx, &vo )
                              : fdgpu_vtile_new_opts( a->device, c->batch_txn, 1UL<<16, 0x5eedUL + (ulong)idx,
                                                      ( mult*c->batch_txn + 64UL ) * 2304UL, FDGPU_SEMANTICS_AVX512, &vo );
  if( !vt ) { fprintf( stderr, "fdgpu_link: tile %d: %s\n", idx, fdgpu_last_error() ); atomic_store( &h->fail, 1 ); return NULL; }
  if( a->svc ) {                               /* where the service's regions lie here: the in dcache, each link's lines */
    int bad = fdgpu_vtile_set_svc_region( vt, 0, l->dcache, h->in_bytes + 4096UL );
    for( ulong q=0; q<Q; q++ ) bad |= fdgpu_vtile_set_svc_region( vt, 1 + (int)q, l->line[q], mc_bytes( h->depth ) );
    if( bad ) { fprintf( stderr, "fdgpu_link: tile %d: service regions\n", idx ); atomic_store( &h->fail, 1 ); fdgpu_vtile_delete( vt ); return NULL; }
  }
  /* zero-copy intake from every producer's link; the overrun check only on unreliable links (a
     reliable producer never reuses a line before the tile's credit passes its pending frags) */
  if( c->zero_copy ) {
    fdgpu_mcache_t const * mcs[ LINK_PROD_MAX ];
    for( ulong q=0; q<Q; q++ ) mcs[q] = c->reliable ? NULL : &l->mc[q];
    if( fdgpu_vtile_set_in_links( vt, mcs, (int)Q ) ) { atomic_store( &h->fail, 1 ); fdgpu_vtile_delete( vt ); return NULL; }
  }
  if( a->svc ) {                               /* served: its GPU context is the service's */
    ulong t_sv = now_ns();
    int r;
    while( !( r = fdgpu_vsvc_ready( a->svc ) ) ) {
      if( atomic_load( &h->fail ) || now_ns() - t_sv > 120000000000UL ) { r = -1; break; }
      usleep( 1000 );
    }
    if( r < 0 ) {
      fprintf( stderr, "fdgpu_link: tile %d: the verify service did not start\n", idx );
      atomic_store( &h->fail, 9 ); fdgpu_vtile_delete( vt ); return NULL;
    }
  }
  atomic_fetch_add( &h->tiles_ready, 1UL );    /* the producers start once every tile has its GPU context */
  {
    ulong t_go = now_ns();                       /* bounded: the producer's process may have died */
    while( !atomic_load_explicit( &h->go, memory_order_acquire ) ) {
      if( atomic_load( &h->fail ) ) { fdgpu_vtile_delete( vt ); return NULL; }
      if( now_ns() - t_go > 180000000000UL ) {
        fprintf( stderr, "fdgpu_link: tile %d waited 180 s for the producer\n", idx );
        atomic_store( &h->fail, 8 ); fdgpu_vtile_delete( vt ); return NULL;
      }
    }
  }
  ulong dcap = 4096UL;
  fdgpu_vtile_done_t * done = (fdgpu_vtile_done_t *)malloc( dcap * sizeof(fdgpu_vtile_done_t) );
  ulong * lh = (ulong *)calloc( LH_N, sizeof(ulong) ), lmax = 0UL, t_last = 0UL;
  uchar * pub = (uchar *)calloc( ( h->n_payload + 7UL ) / 8UL, 1UL );   /* (link_account: payloads this tile published) */
  ulong sigs = 0UL, got = 0UL, lost = 0UL, mine = 0UL;
  link_in_t in[ LINK_PROD_MAX ];
  memset( in, 0, sizeof(in) );
  for( ulong q=0; q<Q; q++ ) { in[q].n = prod_frags( c->n_frags, Q, q ); mine += own_in( 0UL, in[q].n, T, (ulong)idx ); }
  ulong last_prog = ~0UL, t_prog = now_ns(), q0 = 0UL;
  ulong per_link = Q > 1UL ? ( 64UL / Q > 8UL ? 64UL / Q : 8UL ) : 64UL;   /* own frags per link per pass */
  ulong pfl = c->pf_dist > 0 ? (ulong)c->pf_dist : 1UL, pfh = pfl > 1UL ? pfl / 2UL : 1UL;   /* prefetch distances */
  ulong t_hk = 0UL, ns_in = 0UL, ns_after = 0UL, ns_hk = 0UL, ns_idle = 0UL, t_begin = now_ns(), cpu0, iv0;
  ulong const hk_ns = c->hk_ns ? c->hk_ns : 10000UL;
  thread_usage( &cpu0, &iv0 );
  /* FDGPU_LINK_PROF=1: rdtsc section profile (mcache poll, during_frag, prefetch + credit, drain
     after_frags, housekeep after_frags, link_account, credit after a drain, housekeep) */
  int prof = c->prof;
  ulong pc[ 8 ] = { 0 }, c_begin = __rdtsc(), cx = 0UL;
#define PROF_T0()    do { if( prof ) cx = __rdtsc(); } while( 0 )
#define PROF_ADD(i)  do { if( prof ) { ulong cy_ = __rdtsc(); pc[i] += cy_ - cx; cx = cy_; } } while( 0 )
  while( got + lost < mine ) {
    if( atomic_load_explicit( &h->fail, memory_order_relaxed ) ) break;
    ulong t0 = now_ns();
    ulong prog = got;
    for( ulong q=0; q<Q; q++ ) prog += in[q].seq;
    if( prog != last_prog ) { last_prog = prog; t_prog = t0; }
    else if( t0 - t_prog > 30000000000UL ) {                      /* watchdog: 30 s without progress */
      ulong filling = 0, inflight = 0;
      fdgpu_vtile_pipeline_state( vt, &filling, &inflight );
      fprintf( stderr, "fdgpu_link: tile %d stalled: seq[0] %lu got %lu lost %lu / %lu pending %lu filling %lu inflight %lu\n",
               idx, in[0].seq, got, lost, mine, fdgpu_vtile_pending( vt ), filling, inflight );
      atomic_store( &h->fail, 5 ); break;
    }
    /* intake: up to per_link own frags from each link per pass, links in
       turn.  The stem loop reads every seq's line and before_frag drops
       seq % T != idx; with each link's single in-order producer a published
       line of seq implies every earlier seq is published, so the tile reads
       only its own lines (the same frags, without T-1 cross-core line
       transfers per own frag) */
    int drain = 0, all_done = 1, backlog = 0;
    ulong took = 0UL;
    for( ulong qi=0; qi<Q && !drain && !backlog; qi++ ) {
      ulong q = ( q0 + qi ) % Q;
      link_in_t * li = &in[q];
      mc_line_t const * line = l->line[q];
      for( ulong k=0; k<per_link && li->seq < li->n; k++ ) {
        ulong own = li->seq + ( ( (ulong)idx + T - li->seq % T ) % T );   /* next seq with seq % T == idx */
        if( own >= li->n ) { li->seq = li->n; break; }
        mc_line_t const * ln = &line[ own & mask ];
        fdgpu_frag_meta_t m; ulong found;
        PROF_T0();
        int r = mc_poll( ln, own, &m, &found );
        if( r > 0 ) break;                                          /* not yet published */
        PROF_ADD( 0 );
        if( r < 0 ) {
          if( c->reliable ) { atomic_store( &h->fail, 3 ); drain = 1; break; }
          lost += own_in( own, found < li->n ? found : li->n, T, (ulong)idx );   /* overrun: resume there */
          li->seq = found < li->n ? found : li->n;
          continue;
        }
        int rc = fdgpu_vtile_during_frag( vt, q, l->dcache + (ulong)m.chunk * FDGPU_CHUNK_SZ, m.sz, own,
                                          ts_decomp( m.tsorig, t0 ) );   /* the pass's start is "now" to 2^31 ns */
        PROF_ADD( 1 );
        if( rc == -2 ) { drain = 1; li->seq = own; break; }         /* staging full: drain, retry this seq */
        if( rc == FDGPU_VTILE_COPY_BACKLOG ) { backlog = 1; li->seq = own; break; }   /* copies behind: poll them, retry */
        if( rc ) { fprintf( stderr, "fdgpu_link: tile %d during_frag %d\n", idx, rc ); atomic_store( &h->fail, 2 ); drain = 1; break; }
        li->app++; took++;
        /* this tile's next frags of the link are usually published already: start their cold lines,
           software-pipelined -- the mcache line pf_dist own frags ahead, and the record header of the
           frag pf_dist/2 ahead, whose line the prefetch pf_dist/2 iterations ago brought in */
        if( own + pfl*T < li->n ) __builtin_prefetch( &line[ ( own + pfl*T ) & mask ] );
        if( own + pfh*T < li->n ) {
          mc_line_t const * nl = &line[ ( own + pfh*T ) & mask ];
          if( pfh == pfl ) __builtin_prefetch( nl );
          if( atomic_load_explicit( (_Atomic ulong *)&nl->seq, memory_order_relaxed ) == own + pfh*T ) {
            uchar const * pf = l->dcache + (ulong)nl->chunk * FDGPU_CHUNK_SZ;
            __builtin_prefetch( pf ); __builtin_prefetch( pf + 64 );
          }
        }
        li->seq = own + 1UL;
        if( c->reliable && ( li->seq - li->credited >= 64UL || li->seq >= li->n ) ) {   /* batched credit return */
          link_credit( h, (int)q, idx, li, vt ); li->credited = li->seq;
        }
        PROF_ADD( 2 );
      }
      if( li->seq >= li->n && c->reliable && li->credited < li->n ) { link_credit( h, (int)q, idx, li, vt ); li->credited = li->n; }
    }
    q0++;
    for( ulong q=0; q<Q; q++ ) if( in[q].seq < in[q].n ) all_done = 0;
    ulong t1 = now_ns();
    ns_in += t1 - t0;
    if( !took && !drain ) ns_idle += t1 - t0;
    if( atomic_load_explicit( &h->fail, memory_order_relaxed ) ) break;
    if( drain || ( all_done && fdgpu_vtile_pending( vt ) ) ) {
      fdgpu_vtile_copy( vt, 0 );                                     /* the frags taken are copied while it waits */
      PROF_T0();
      ulong n = fdgpu_vtile_after_frags( vt, done, dcap, 1 );
      PROF_ADD( 3 );
      link_trace( l, idx, vt, done, n );
      link_account( l, idx, done, n, &sigs, lh, &lmax, &t_last, in, pub ); got += n;
      PROF_ADD( 5 );
      if( c->reliable && c->zero_copy ) for( ulong q=0; q<Q; q++ ) link_credit( h, (int)q, idx, &in[q], vt );
      PROF_ADD( 6 );
      ns_after += now_ns() - t1;
      continue;
    }
    /* housekeeping: launch / drain at most every 10 us while frags flow
       (the HIP runtime calls behind them take locks shared by all tiles) */
    if( backlog || t1 - t_hk >= hk_ns ) {
      t_hk = t1;
      PROF_T0();
      fdgpu_vtile_housekeep( vt, c->max_inflight );                 /* adaptive batching */
      PROF_ADD( 7 );
      ulong t2 = now_ns();
      PROF_T0();
      ulong n = fdgpu_vtile_after_frags( vt, done, dcap, 0 );
      PROF_ADD( 4 );
      link_trace( l, idx, vt, done, n );
      link_account( l, idx, done, n, &sigs, lh, &lmax, &t_last, in, pub ); got += n;
      PROF_ADD( 5 );
      if( c->reliable && c->zero_copy ) for( ulong q=0; q<Q; q++ ) link_credit( h, (int)q, idx, &in[q], vt );
      PROF_ADD( 6 );
      ns_hk += t2 - t1; ns_after += now_ns() - t2;
    }
  }
  ulong t_end = now_ns();
  link_res_t * r = &l->res[idx];
  double cyc_per_ns = (double)( __rdtsc() - c_begin ) / (double)( t_end - t_begin + 1UL );
  for( int i=0; i<8; i++ ) r->prof[i] = prof ? (ulong)( (double)pc[i] / cyc_per_ns ) : 0UL;
#undef PROF_T0
#undef PROF_ADD
  r->verdicts = got; r->lost = lost; r->overruns = fdgpu_vtile_overruns( vt );
  r->sigs = sigs; r->t_last = t_last; r->lmax = lmax;
  fdgpu_vtile_metrics( vt, r->metrics );
  r->ns[0] = ns_in; r->ns[1] = ns_after; r->ns[2] = ns_hk; r->ns[3] = t_end - t_begin; r->ns_idle = ns_idle;
  fdgpu_vtile_gpu_metrics( vt, &r->gm );
  r->device = (ulong)a->device;
  ulong cpu1, iv1;
  thread_usage( &cpu1, &iv1 );
  r->cpu_ns = cpu1 - cpu0; r->wall_ns = t_end - t_begin; r->nivcsw = iv1 - iv0; r->cpu = a->cpu;
  r->gpu_open = proc_has_gpu_open() > 0;
  memcpy( l->hist + (ulong)idx * LH_N, lh, LH_N * sizeof(ulong) );
  /* (a served tile is counted done by its service's process, once it has added the GPU side's metrics) */
  if( !a->svc ) atomic_fetch_add_explicit( &h->tiles_done, 1UL, memory_order_release );
  free( done ); free( lh ); free( pub );
  fdgpu_vtile_delete( vt );
  return NULL;
}

/* Each process runs its tiles (i % G == proc) and, with run_producer, its
   producers (q % G == proc). */
static int link_run_svc( fdgpu_link_t * l, int proc, int device, int run_producer );

int
fdgpu_link_run( fdgpu_link_t * l, int proc, int device, int run_producer ) {
  link_hdr_t * h = l->h;
  fdgpu_stream_cfg_t const * c = &h->cfg;
  if( proc < 0 || proc >= c->gpus ) return -1;
  if( c->svc ) return link_run_svc( l, proc, device, run_producer );
  if( c->zero_copy && !l->registered ) {
    if( fdgpu_host_register( l->dcache, h->in_bytes + 4096UL ) ) { atomic_store( &h->fail, 7 ); return -3; }
    for( int q=0; q<c->producers; q++ )          /* the gather re-reads each frag's line after its copy */
      if( fdgpu_host_register( l->line[q], mc_bytes( h->depth ) ) ) {
        /* undo what was registered: fdgpu_link_delete unregisters only a complete registration */
        while( q-- > 0 ) fdgpu_host_unregister( l->line[q] );
        fdgpu_host_unregister( l->dcache );
        atomic_store( &h->fail, 7 ); return -3;
      }
    l->registered = 1;
  }
  pthread_t prod[ LINK_PROD_MAX ], th[ LINK_TILE_MAX ];
  link_tile_arg_t args[ LINK_TILE_MAX ];
  link_prod_arg_t pargs[ LINK_PROD_MAX ];
  memset( args, 0, sizeof(args) );               /* (svc NULL: tiles with engine contexts of their own) */
  int mine[ LINK_TILE_MAX ], myq[ LINK_PROD_MAX ], np = 0;
  int nt = fdgpu_link_tiles_of( c->tiles, c->gpus, proc, mine );   /* tile i drives GPU i % G: this process's tiles */
  if( run_producer ) for( int q=0; q<c->producers; q++ ) if( q % c->gpus == proc ) myq[np++] = q;
  int cpus[ ( 2 + FDGPU_VTILE_COPY_THREADS_MAX )*LINK_TILE_MAX + LINK_PROD_MAX ];
  int nl = c->launcher ? nt : 0;                 /* the tiles' launch threads: a core each, after the tiles' */
  int H = c->zero_copy && c->copy_threads > 0 ? ( c->copy_threads < FDGPU_VTILE_COPY_THREADS_MAX ? c->copy_threads
                                                                                                  : FDGPU_VTILE_COPY_THREADS_MAX ) : 0;
  int ncpu = link_pick_cpus( device, proc, nt + np + nl + nt*H, np + nt, cpus, 1 );   /* ... and their copy threads, after those */
  link_place_producers( c, myq, np, cpus, ncpu, fdgpu_device_numa_node( device ) );
  if( getenv( "FDGPU_LINK_VERBOSE" ) ) {
    fprintf( stderr, "fdgpu_link: proc %d device %d numa %d producers %d tiles %d cpus:", proc, device,
             fdgpu_device_numa_node( device ), np, nt );
    for( int i=0; i<ncpu; i++ ) fprintf( stderr, " %d", cpus[i] );
    fprintf( stderr, "\n" );
  }
  for( int t=0; t<nt; t++ ) {
    args[t].l = l; args[t].idx = mine[t]; args[t].device = device;
    args[t].cpu = np + t < ncpu ? cpus[ np + t ] : -1;
    args[t].lcpu = nl && np + nt + t < ncpu ? cpus[ np + nt + t ] : -1;
    for( int i=0; i<FDGPU_VTILE_COPY_THREADS_MAX; i++ ) {
      int j = np + nt + nl + t*H + i;
      args[t].ccpu[i] = i < H && j < ncpu ? cpus[j] : -1;
    }
    pthread_create( &th[t], NULL, link_tile, &args[t] );
  }
  for( int i=0; i<np; i++ ) {
    pargs[i].l = l; pargs[i].q = myq[i]; pargs[i].cpu = i < ncpu ? cpus[i] : -1;
    pthread_create( &prod[i], NULL, link_producer, &pargs[i] );
  }
  for( int i=0; i<np; i++ ) pthread_join( prod[i], NULL );
  for( int t=0; t<nt; t++ ) pthread_join( th[t], NULL );
  int rc = (int)atomic_load( &h->fail );
  return rc ? -rc - 10 : 0;
}

/* Served tiles (cfg.svc): each tile of this process's GPU runs as a process of its own -- the tile program
   (fdgpu_tile, fd_vtile_main.c), started here, which joins the link and the service segment by their files and
   runs link_tile's loop with no GPU context (fdgpu_link_run_tile) -- and this process is their verify service
   (fdgpu_vsvc_*, one thread) and runs its producers.  The GPU side's metrics (batches, latency histogram,
   gathers, phases) are the service's: they are added to this process's first tile's results before its tiles
   are counted done. */
typedef struct { fdgpu_vsvc_t * svc; link_hdr_t * h; int device, cpu; _Atomic int stop; } link_svc_arg_t;

static void * link_svc_main( void * _a ) {
  link_svc_arg_t * a = (link_svc_arg_t *)_a;
  link_pin( a->cpu );
  if( fdgpu_vsvc_start( a->svc, a->device ) ) { atomic_store( &a->h->fail, 7 ); return NULL; }
  while( !atomic_load_explicit( &a->stop, memory_order_acquire ) )
    if( !fdgpu_vsvc_poll( a->svc ) ) _mm_pause();
  return NULL;
}

/* the tile program, next to this library */
static int tile_prog_path( char * out, ulong n ) {
  Dl_info di;
  if( !dladdr( (void *)fdgpu_link_run_tile, &di ) || !di.dli_fname ) return -1;
  char const * sl = strrchr( di.dli_fname, '/' );
  int dl = sl ? (int)( sl - di.dli_fname ) : 1;
  if( snprintf( out, n, "%.*s/fdgpu_tile", dl, sl ? di.dli_fname : "." ) >= (int)n ) return -1;
  return access( out, X_OK ) ? -1 : 0;
}

extern char ** environ;

static int
link_run_svc( fdgpu_link_t * l, int proc, int device, int run_producer ) {
  link_hdr_t * h = l->h;
  fdgpu_stream_cfg_t const * c = &h->cfg;
  int mine[ LINK_TILE_MAX ], myq[ LINK_PROD_MAX ], np = 0;
  int nt = fdgpu_link_tiles_of( c->tiles, c->gpus, proc, mine );
  if( nt < 1 || nt > FDGPU_VSVC_CLIENT_MAX || !l->shared ) return -1;
  char prog[ 512 ];
  if( tile_prog_path( prog, sizeof(prog) ) ) { fprintf( stderr, "fdgpu_link: the tile program fdgpu_tile is missing\n" ); return -1; }
  if( run_producer ) for( int q=0; q<c->producers; q++ ) if( q % c->gpus == proc ) myq[np++] = q;
  int nl = c->launcher ? 1 : 0;
  int H = c->zero_copy && c->copy_threads > 0 ? ( c->copy_threads < FDGPU_VTILE_COPY_THREADS_MAX ? c->copy_threads
                                                                                                  : FDGPU_VTILE_COPY_THREADS_MAX ) : 0;
  /* CPUs: producers, tiles, the service, its launch thread, the tiles' copy threads */
  int cpus[ ( 2 + FDGPU_VTILE_COPY_THREADS_MAX )*LINK_TILE_MAX + LINK_PROD_MAX + 2 ];
  int ncpu = link_pick_cpus( device, proc, np + nt + 1 + nl + nt*H, np + nt, cpus, 1 );
  link_place_producers( c, myq, np, cpus, ncpu, fdgpu_device_numa_node( device ) );
  int svc_cpu = np + nt < ncpu ? cpus[ np + nt ] : -1, lcpu = nl && np + nt + 1 < ncpu ? cpus[ np + nt + 1 ] : -1;
  if( getenv( "FDGPU_LINK_VERBOSE" ) ) {
    fprintf( stderr, "fdgpu_link: served: proc %d device %d producers %d tiles %d service cpu %d cpus:", proc, device, np, nt, svc_cpu );
    for( int i=0; i<ncpu; i++ ) fprintf( stderr, " %d", cpus[i] );
    fprintf( stderr, "\n" );
  }
  ulong mult = c->out_mult ? c->out_mult : 6UL;
  fdgpu_vsvc_cfg_t sc;
  memset( &sc, 0, sizeof(sc) );
  sc.clients = nt; sc.out_dcache_bytes = ( mult*c->batch_txn + 64UL ) * 2304UL; sc.batch_txn = c->batch_txn;
  sc.max_inflight = c->max_inflight; sc.semantics = FDGPU_SEMANTICS_AVX512; sc.nctx = c->nctx; sc.small_max = c->small_max;
  sc.min_batch = c->min_batch; sc.copy_wait_ns = c->copy_wait_ns; sc.copy_min = c->copy_min; sc.gather_cus = c->gather_cus;
  sc.cu_split = c->cu_split; sc.cu_exclusive = c->cu_exclusive; sc.lat_share = c->lat_share;
  sc.launcher = c->launcher; sc.launcher_core = lcpu >= 0 ? lcpu + 1 : 0;
  char spath[ 300 ];
  snprintf( spath, sizeof(spath), "%s.svc%d", l->path, proc );
  fdgpu_vsvc_t * svc = fdgpu_vsvc_new( spath, &sc );
  if( !svc ) { fprintf( stderr, "fdgpu_link: service segment %s\n", spath ); atomic_store( &h->fail, 7 ); return -3; }
  /* the service's regions: the in dcache (0) and each producer's mcache lines (1 + q) */
  int bad = fdgpu_vsvc_add_region( svc, 0, l->dcache, h->in_bytes + 4096UL );
  for( int q=0; q<c->producers; q++ ) bad |= fdgpu_vsvc_add_region( svc, 1 + q, l->line[q], mc_bytes( h->depth ) );
  if( bad ) { fdgpu_vsvc_delete( svc ); atomic_store( &h->fail, 7 ); return -3; }
  /* the tile processes: fdgpu_tile <link> <service> <tile> <cpu> [copy thread cpus] */
  pid_t pid[ LINK_TILE_MAX ];
  int nspawn = 0;
  for( int t=0; t<nt; t++ ) {
    char a_tile[ 16 ], a_cpu[ 16 ], a_cc[ FDGPU_VTILE_COPY_THREADS_MAX ][ 16 ];
    char * argv[ 6 + FDGPU_VTILE_COPY_THREADS_MAX ];
    int na = 0;
    snprintf( a_tile, sizeof(a_tile), "%d", mine[t] );
    snprintf( a_cpu, sizeof(a_cpu), "%d", np + t < ncpu ? cpus[ np + t ] : -1 );
    argv[na++] = prog; argv[na++] = l->path; argv[na++] = spath; argv[na++] = a_tile; argv[na++] = a_cpu;
    for( int i=0; i<H; i++ ) {
      int j = np + nt + 1 + nl + t*H + i;
      snprintf( a_cc[i], sizeof(a_cc[i]), "%d", j < ncpu ? cpus[j] : -1 );
      argv[na++] = a_cc[i];
    }
    argv[na] = NULL;
    pid_t p;
    if( posix_spawn( &p, prog, NULL, NULL, argv, environ ) ) { atomic_store( &h->fail, 12 ); break; }
    pid[ nspawn++ ] = p;
  }
  /* this process: the service, then the producers */
  link_svc_arg_t sa;
  memset( &sa, 0, sizeof(sa) );
  sa.svc = svc; sa.h = h; sa.device = device; sa.cpu = svc_cpu;
  pthread_t sth, prod[ LINK_PROD_MAX ];
  link_prod_arg_t pargs[ LINK_PROD_MAX ];
  int sth_ok = !pthread_create( &sth, NULL, link_svc_main, &sa );
  if( !sth_ok ) atomic_store( &h->fail, 7 );
  for( int i=0; i<np; i++ ) {
    pargs[i].l = l; pargs[i].q = myq[i]; pargs[i].cpu = i < ncpu ? cpus[i] : -1;
    pthread_create( &prod[i], NULL, link_producer, &pargs[i] );
  }
  /* wait for the tile processes (a tile that dies fails the run: the others see h->fail and stop) */
  int left = nspawn;
  while( left ) {
    for( int t=0; t<nspawn; t++ ) {
      if( pid[t] < 0 ) continue;
      int st = 0;
      pid_t p = waitpid( pid[t], &st, WNOHANG );
      if( p == 0 ) continue;
      pid[t] = -1; left--;
      if( p < 0 || !WIFEXITED( st ) || WEXITSTATUS( st ) ) {
        fprintf( stderr, "fdgpu_link: served tile process %d ended with status %d\n", t, st );
        if( !atomic_load( &h->fail ) ) atomic_store( &h->fail, 13 );
      }
    }
    if( left ) usleep( 1000 );
  }
  for( int i=0; i<np; i++ ) pthread_join( prod[i], NULL );
  atomic_store_explicit( &sa.stop, 1, memory_order_release );
  if( sth_ok ) pthread_join( sth, NULL );
  /* the GPU side's metrics into this process's first tile's results, then its tiles are done */
  fdgpu_vsvc_stats_t ss;
  fdgpu_vsvc_stats( svc, &ss );
  fdgpu_vtile_gpu_metrics_t * gm = &l->res[ mine[0] ].gm;
  gm->batches += ss.gm.batches; gm->batch_txns += ss.gm.batch_txns;
  if( ss.gm.inflight_max > gm->inflight_max ) gm->inflight_max = ss.gm.inflight_max;
  for( ulong k=0; k<FDGPU_VTILE_LAT_BUCKETS; k++ ) gm->lat_hist[k] += ss.gm.lat_hist[k];
  gm->launch_ns += ss.gm.launch_ns; gm->copies += ss.gm.copies;
  for( int k=0; k<8; k++ ) gm->gather_gpu[k] = ss.gm.gather_gpu[k];
  for( int k=0; k<9; k++ ) gm->phase[k] = ss.gm.phase[k];
  for( int k=0; k<6; k++ ) gm->launcher[k] = ss.gm.launcher[k];
  gm->faults += ss.gm.faults;
  l->svc_stats = ss;
  l->svc_cpu = svc_cpu;
  atomic_fetch_add_explicit( &h->tiles_done, (ulong)nt, memory_order_release );
  fdgpu_vsvc_delete( svc );
  int rc = (int)atomic_load( &h->fail );
  return rc ? -rc - 10 : 0;
}

/* the tile program's body: tile `tile` of a shared link, served by the service segment at svc_path (made by the
   process that runs the tile's GPU, proc = tile % G).  No GPU call. */
int
fdgpu_link_run_tile( fdgpu_link_t * l, int tile, char const * svc_path, int cpu, int const * copy_cpus, int ncopy ) {
  link_hdr_t * h = l->h;
  fdgpu_stream_cfg_t const * c = &h->cfg;
  if( tile < 0 || tile >= c->tiles ) return -1;
  int proc = tile % c->gpus, mine[ LINK_TILE_MAX ];
  int nt = fdgpu_link_tiles_of( c->tiles, c->gpus, proc, mine ), client = -1;
  for( int i=0; i<nt; i++ ) if( mine[i] == tile ) client = i;
  if( client < 0 ) return -1;
  fdgpu_vsvc_t * svc = fdgpu_vsvc_join( svc_path, 60. );
  if( !svc ) { fprintf( stderr, "fdgpu_tile %d: no service segment %s\n", tile, svc_path ); atomic_store( &h->fail, 9 ); return -9; }
  link_tile_arg_t a;
  memset( &a, 0, sizeof(a) );
  a.l = l; a.idx = tile; a.device = -1; a.cpu = cpu; a.lcpu = -1;
  for( int i=0; i<FDGPU_VTILE_COPY_THREADS_MAX; i++ ) a.ccpu[i] = copy_cpus && i < ncopy ? copy_cpus[i] : -1;
  a.svc = svc; a.client = client;
  link_tile( &a );
  fdgpu_vsvc_delete( svc );
  int rc = (int)atomic_load( &h->fail );
  return rc ? -rc - 10 : 0;
}

int
fdgpu_link_svc_stats( fdgpu_link_t const * l, fdgpu_vsvc_stats_t * out, int * svc_cpu ) {
  *out = l->svc_stats;
  if( svc_cpu ) *svc_cpu = l->svc_cpu;
  return 0;
}

int
fdgpu_link_result( fdgpu_link_t * l, double timeout_s, fdgpu_stream_stats_t * st ) {
  link_hdr_t * h = l->h;
  fdgpu_stream_cfg_t const * c = &h->cfg;
  ulong T = (ulong)c->tiles, t0 = now_ns(), lim = (ulong)( timeout_s * 1e9 );
  while( atomic_load_explicit( &h->tiles_done, memory_order_acquire ) < T ) {
    if( atomic_load( &h->fail ) ) return -(int)atomic_load( &h->fail ) - 10;
    if( now_ns() - t0 > lim ) return -2;
    usleep( 1000 );
  }
  memset( st, 0, sizeof(*st) );
  for( int q=0; q<4; q++ ) st->prod_cpu[q] = -1L;
  ulong * lh = (ulong *)calloc( LH_N, sizeof(ulong) );
  if( !lh ) return -3;
  ulong t_end = 0UL, lmax = 0UL;
  for( ulong i=0; i<T; i++ ) {
    link_res_t const * r = &l->res[i];
    st->sigs += r->sigs; st->verdicts += r->verdicts; st->lost += r->lost; st->overruns += r->overruns;
    for( int k=0; k<5; k++ ) st->metrics[k] += r->metrics[k];
    for( int k=0; k<4; k++ ) st->tile_ns[k] += r->ns[k];
    st->batches += r->gm.batches; st->batch_txns += r->gm.batch_txns;
    if( r->gm.inflight_max > st->inflight_max ) st->inflight_max = r->gm.inflight_max;
    for( ulong k=0; k<FDGPU_VTILE_LAT_BUCKETS; k++ ) st->gpu_lat_hist[k] += r->gm.lat_hist[k];
    st->gpu_wait_ns += r->gm.wait_ns; st->poll_ns += r->gm.poll_ns; st->after_ns += r->gm.after_ns;
    st->launch_ns += r->gm.launch_ns;
    st->copies += r->gm.copies; st->copy_lat_n += r->gm.copy_lat_n; st->copy_lat_ns_sum += r->gm.copy_lat_ns_sum;
    if( r->gm.copy_lat_ns_max > st->copy_lat_ns_max ) st->copy_lat_ns_max = r->gm.copy_lat_ns_max;
    for( int k=0; k<8; k++ ) {
      if( k == 2 || k == 4 || k == 6 ) { if( r->gm.gather_gpu[k] > st->gather_gpu[k] ) st->gather_gpu[k] = r->gm.gather_gpu[k]; }
      else st->gather_gpu[k] += r->gm.gather_gpu[k];
    }
    for( int k=0; k<9; k++ ) {
      if( k == 2 || k == 4 || k == 6 ) { if( r->gm.phase[k] > st->phase[k] ) st->phase[k] = r->gm.phase[k]; }
      else st->phase[k] += r->gm.phase[k];
    }
    st->copy_backlog += r->gm.copy_backlog;
    st->launcher[0] += r->gm.launcher[0]; st->launcher[1] += r->gm.launcher[1]; st->launcher[3] += r->gm.launcher[3];
    st->launcher[5] += r->gm.launcher[5];
    if( r->gm.launcher[2] > st->launcher[2] ) st->launcher[2] = r->gm.launcher[2];
    if( r->gm.launcher[4] > st->launcher[4] ) st->launcher[4] = r->gm.launcher[4];
    for( int k=0; k<4; k++ ) st->host_copy[k] += r->gm.host_copy[k];
    st->tiles_gpu_open += r->gpu_open;
    st->tile_idle_ns += r->ns_idle;
    st->tile_cpu_ns += r->cpu_ns; st->tile_wall_ns += r->wall_ns; st->tile_nivcsw += r->nivcsw;
    double share = r->wall_ns ? (double)r->cpu_ns / (double)r->wall_ns : 1.;
    if( i == 0 || share < st->tile_cpu_share_min ) st->tile_cpu_share_min = share;
    if( i < 8 ) st->tile_cpu[i] = r->cpu;
    for( int k=0; k<8; k++ ) st->prof_ns[k] += r->prof[k];
    if( r->t_last > t_end ) t_end = r->t_last;
    if( r->lmax > lmax ) lmax = r->lmax;
    for( ulong k=0UL; k<LH_N; k++ ) lh[k] += l->hist[ i*LH_N + k ];
  }
  ulong prod_end = 0UL;
  for( int q=0; q<c->producers; q++ ) {
    if( h->prod_end[q] > prod_end ) prod_end = h->prod_end[q];
    st->prod_wait_ns += h->prod_wait_ns[q];
    st->prod_cpu_ns += h->prod_cpu_ns[q]; st->prod_wall_ns += h->prod_wall_ns[q]; st->prod_nivcsw += h->prod_nivcsw[q];
    if( q < 4 ) st->prod_cpu[q] = h->prod_cpu[q];
  }
  st->seconds = t_end > h->t_start ? (double)( t_end - h->t_start ) * 1e-9 : 0.;
  st->prod_seconds = prod_end > h->t_start ? (double)( prod_end - h->t_start ) * 1e-9 : 0.;
  st->frags = c->n_frags;
  st->published = st->metrics[4];
  st->frags_per_s = st->seconds > 0. ? (double)st->verdicts / st->seconds : 0.;
  st->sigs_per_s  = st->seconds > 0. ? (double)st->sigs / st->seconds : 0.;
  ulong tot = 0UL;
  for( ulong k=0UL; k<LH_N; k++ ) tot += lh[k];
  st->lat_p50_us = tot ? lh_quantile( lh, tot, 0.50 ) * 1e-3 : 0.;
  st->lat_p99_us = tot ? lh_quantile( lh, tot, 0.99 ) * 1e-3 : 0.;
  st->lat_max_us = (double)lmax * 1e-3;
  st->tiles = c->tiles; st->gpus = c->gpus;
  free( lh );
  return 0;
}

/* private link, producers + every tile in this process on one device (G = 1) */
int
fdgpu_stream_run( int device, fdgpu_stream_cfg_t const * cfg, uchar const * payload, unsigned const * off,
                  unsigned short const * sz, ulong n_payload, ulong mcache_depth, fdgpu_stream_stats_t * st ) {
  fdgpu_stream_cfg_t c = *cfg;
  c.gpus = 1;
  /* served tiles join the link from processes of their own: a file then */
  static _Atomic ulong seq = 0UL;
  char path[ 128 ];
  if( c.svc ) snprintf( path, sizeof(path), "/dev/shm/fdgpu_stream_%d_%lu", (int)getpid(), atomic_fetch_add( &seq, 1UL ) );
  fdgpu_link_t * l = fdgpu_link_new( c.svc ? path : NULL, &c, payload, off, sz, n_payload, mcache_depth );
  if( !l ) return -1;
  int rc = fdgpu_link_run( l, 0, device, 1 );
  if( !rc ) rc = fdgpu_link_result( l, 60., st );
  fdgpu_link_delete( l );
  if( c.svc ) unlink( path );
  return rc;
}

int
fdgpu_stream_bench( int device, uchar const * payload, unsigned const * off, unsigned short const * sz, ulong n_payload,
                    ulong n_frags, int tiles, ulong batch_txn, ulong max_inflight, ulong mcache_depth, double rate_fps,
                    int zero_copy, fdgpu_stream_stats_t * st ) {
  fdgpu_stream_cfg_t c;
  memset( &c, 0, sizeof(c) );
  c.n_frags = n_frags; c.batch_txn = batch_txn; c.max_inflight = max_inflight ? max_inflight : 2UL; c.rate_fps = rate_fps;
  c.tiles = tiles; c.gpus = 1; c.zero_copy = zero_copy; c.reliable = 1; c.producers = 1;
  return fdgpu_stream_run( device, &c, payload, off, sz, n_payload, mcache_depth, st );
}
