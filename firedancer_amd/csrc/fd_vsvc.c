/* fd_vsvc.c -- the verify service: one process per GPU that owns the GPU and verifies the frags of
   several verify-tile processes (include/fd_verify_gpu.h, fdgpu_vsvc_*; the shared segment's layout is
   fd_vsvc_private.h).  Host C over the engine (libfdgpu_ed25519.so).

   The reference runs each verify tile as a process of its own (src/disco/topo/fd_topo_run.c:66-153,
   six by default, src/app/fdctl/config/default.toml:788).  Here those processes make no GPU call: each
   hands its frags to this service through a request ring, and the service batches the frags of all of
   them into one stream of GPU batches -- what one tile with engine contexts of its own does for its
   frags alone (fd_verify_gpu.c: the same adaptive launch, staggered contexts, early copies, CU
   reservations) -- then writes each verdict back into its tile's completion ring, in the tile's order.
   A batch mixes tiles: each record is copied from the tile's in link into the GPU and back into that
   tile's out dcache (fdgpu_ed25519_submit_raw_gather_to), and its HA dedup tag is computed with that
   tile's secure seed (fd_verify_tile.c:166; FDGPU_GATHER_SEED). */

#define _GNU_SOURCE
#include "fd_vsvc_private.h"
#include "../../include/fd_ed25519_gpu.h"

#include <fcntl.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <time.h>
#include <unistd.h>
#include <x86intrin.h>

typedef unsigned long ulong;
typedef unsigned char uchar;

static ulong sv_now( void ) {
  struct timespec ts; clock_gettime( CLOCK_MONOTONIC, &ts );
  return (ulong)ts.tv_sec * 1000000000UL + (ulong)ts.tv_nsec;
}
static ulong sv_pow2_up( ulong x ) { ulong p = 1UL; while( p < x ) p <<= 1; return p; }

#define SV_HUGE          (2UL << 20)
#define SV_RESERVE_MAX   ( FDGPU_TXNM_HDR_SZ + 1232UL + 2UL + 852UL )   /* header + MTU payload + fd_txn_t (as a tile) */
#define SV_RCHUNK        ( ( ( SV_RESERVE_MAX + 127UL ) >> 7 ) << 1 )

/* ---- the segment ---------------------------------------------------------- */

/* frags a tile with an out dcache of out_sz bytes can have pending (fdgpu_vtile_new_opts' pend_cap) */
static ulong sv_pend_cap( ulong out_sz ) { return ( ( out_sz / FDGPU_CHUNK_SZ ) & ~1UL ) / SV_RCHUNK - 2UL; }

fdgpu_vsvc_t *
fdgpu_vsvc_new( char const * path, fdgpu_vsvc_cfg_t const * cfg ) {
  if( !cfg || cfg->clients < 1 || cfg->clients > FDGPU_VSVC_CLIENT_MAX || !cfg->batch_txn ||
      cfg->out_dcache_bytes < 8UL*SV_RESERVE_MAX || ( path && strlen( path ) >= 256 ) ) return NULL;
  ulong C = (ulong)cfg->clients;
  ulong out_sz = cfg->out_dcache_bytes & ~127UL;
  ulong ring = sv_pow2_up( sv_pend_cap( out_sz ) + 2UL );
  ulong o = ( sizeof(vsvc_hdr_t) + 4095UL ) & ~4095UL;
  ulong off_req[ FDGPU_VSVC_CLIENT_MAX ], off_cpl[ FDGPU_VSVC_CLIENT_MAX ], off_out[ FDGPU_VSVC_CLIENT_MAX ];
  for( ulong c=0; c<C; c++ ) {
    off_req[c] = o; o += ring * sizeof(vsvc_req_t);
    off_cpl[c] = o; o += ring * sizeof(vsvc_cpl_t);
    o = ( o + 4095UL ) & ~4095UL;
  }
  o = ( o + SV_HUGE - 1UL ) & ~( SV_HUGE - 1UL );
  for( ulong c=0; c<C; c++ ) { off_out[c] = o; o += ( out_sz + SV_HUGE - 1UL ) & ~( SV_HUGE - 1UL ); }
  ulong total = o;
  fdgpu_vsvc_t * s = (fdgpu_vsvc_t *)calloc( 1, sizeof(fdgpu_vsvc_t) );
  if( !s ) return NULL;
  uchar * base;
  if( path ) {
    int fd = open( path, O_RDWR | O_CREAT | O_EXCL, 0600 );
    if( fd < 0 ) { free( s ); return NULL; }
    if( ftruncate( fd, (off_t)total ) ) { close( fd ); unlink( path ); free( s ); return NULL; }
    base = (uchar *)mmap( NULL, total, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0 );
    close( fd );
    if( base == MAP_FAILED ) { unlink( path ); free( s ); return NULL; }
    strcpy( s->path, path );
  } else {
    /* anonymous shared memory: tile processes forked from this one see the same pages */
    base = (uchar *)mmap( NULL, total, PROT_READ | PROT_WRITE, MAP_SHARED | MAP_ANONYMOUS, -1, 0 );
    if( base == MAP_FAILED ) { free( s ); return NULL; }
  }
  (void)madvise( base, total, MADV_HUGEPAGE );   /* shmem: where shmem_enabled allows (the out dcaches are 2 MiB aligned) */
  s->h = (vsvc_hdr_t *)base; s->base = base; s->sz = total; s->creator = 1; s->cfg = *cfg;
  vsvc_hdr_t * h = s->h;
  memset( (void *)h, 0, sizeof(vsvc_hdr_t) );
  h->total_sz = total; h->clients = (int)C; h->ring_cap = ring; h->out_sz = out_sz;
  s->nclients = (int)C; s->ring = ring; s->out_sz = out_sz;
  for( ulong c=0; c<C; c++ ) {
    vsvc_client_t * k = &h->client[c];
    k->off_req = off_req[c]; k->off_cpl = off_cpl[c]; k->off_out = off_out[c]; k->ring_cap = ring; k->out_sz = out_sz;
    s->off_req[c] = off_req[c]; s->off_cpl[c] = off_cpl[c]; s->off_out[c] = off_out[c];
  }
  atomic_store_explicit( &h->joined, 1UL, memory_order_relaxed );
  atomic_store_explicit( &h->magic, VSVC_MAGIC, memory_order_release );
  return s;
}

fdgpu_vsvc_t *
fdgpu_vsvc_join( char const * path, double timeout_s ) {
  if( !path || strlen( path ) >= 256 ) return NULL;
  ulong t0 = sv_now(), lim = (ulong)( timeout_s * 1e9 );
  for(;;) {
    int fd = open( path, O_RDWR );
    if( fd >= 0 ) {
      struct stat st;
      if( !fstat( fd, &st ) && (ulong)st.st_size >= sizeof(vsvc_hdr_t) ) {
        vsvc_hdr_t * h = (vsvc_hdr_t *)mmap( NULL, sizeof(vsvc_hdr_t), PROT_READ, MAP_SHARED, fd, 0 );
        if( h != MAP_FAILED ) {
          int ok = atomic_load_explicit( &h->magic, memory_order_acquire ) == VSVC_MAGIC;
          ulong total = h->total_sz;
          munmap( (void *)h, sizeof(vsvc_hdr_t) );
          if( ok && (ulong)st.st_size >= total ) {
            uchar * base = (uchar *)mmap( NULL, total, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0 );
            close( fd );
            if( base == MAP_FAILED ) return NULL;
            fdgpu_vsvc_t * s = (fdgpu_vsvc_t *)calloc( 1, sizeof(fdgpu_vsvc_t) );
            if( !s ) { munmap( base, total ); return NULL; }
            s->h = (vsvc_hdr_t *)base; s->base = base; s->sz = total; strcpy( s->path, path );
            /* the rings' pages now (a tile writes requests and reads completions from its first frag on; the
               out dcaches, which only the GPU and the tile's readers touch, are left to fault in) */
            for( int c=0; c<s->h->clients; c++ ) {
              vsvc_client_t const * k = &s->h->client[c];
              ulong lo = k->off_req & ~4095UL, hi = k->off_cpl + k->ring_cap * sizeof(vsvc_cpl_t);
              (void)madvise( base + lo, hi - lo, MADV_WILLNEED );
              for( ulong o=lo; o<hi; o+=4096UL ) (void)*(volatile uchar const *)( base + o );
            }
            atomic_fetch_add( &s->h->joined, 1UL );
            return s;
          }
        }
      }
      close( fd );
    }
    if( sv_now() - t0 > lim ) return NULL;
    usleep( 2000 );
  }
}

int
fdgpu_vsvc_add_region( fdgpu_vsvc_t * s, int id, void * base, ulong sz ) {
  if( !s || !s->creator || s->started || id < 0 || id >= FDGPU_VSVC_RGN_MAX || !base || !sz ) return -1;
  s->rgn_host[id] = (uchar *)base; s->rgn_sz[id] = sz; s->h->rgn_sz[id] = sz;
  return 0;
}

int  fdgpu_vsvc_ready( fdgpu_vsvc_t const * s ) { return atomic_load_explicit( &s->h->ready, memory_order_acquire ); }
void fdgpu_vsvc_stop( fdgpu_vsvc_t * s ) { atomic_store_explicit( &s->h->stop, 1, memory_order_release ); }
ulong fdgpu_vsvc_pending( fdgpu_vsvc_t const * s ) { return s->ptail - s->phead; }

/* ---- the GPU side ----------------------------------------------------------- */

/* one engine context of the service, set up as a verify tile sets up its own (fd_verify_gpu.c vt_ctx_new) */
static fdgpu_ed25519_ctx_t *
sv_ctx_new( fdgpu_vsvc_t * s, int k ) {
  ulong b = s->cfg.batch_txn;
  fdgpu_ed25519_ctx_t * c = fdgpu_ed25519_ctx_new( s->device, b, 16UL*b, b*2304UL + 1024UL, s->cfg.semantics );
  if( !c ) return NULL;
  ulong sm = fdgpu_ed25519_set_small_batch_max( c, 0UL );
  fdgpu_ed25519_set_small_batch_max( c, s->cfg.small_max ? s->cfg.small_max : ( sm < b/2UL ? sm : b/2UL ) );
  if( fdgpu_ed25519_set_dedup_seeds( c, s->seeds, s->nclients ) ) goto fail;
  unsigned parts = s->cfg.cu_split ? (unsigned)s->nctx : 1u, part = s->cfg.cu_split ? (unsigned)k : 0u;
  if( s->cfg.gather_cus && fdgpu_ed25519_reserve_cus( c, s->cfg.gather_cus, part, parts ) ) goto fail;
  int excl = s->cfg.cu_exclusive ? s->cfg.cu_exclusive : ( fdgpu_ed25519_get_cu_exclusive( c ) ? 0 : 1 );
  if( excl > 0 && fdgpu_ed25519_set_cu_exclusive( c, excl ) ) goto fail;
  unsigned share = s->cfg.lat_share > 0 ? (unsigned)s->cfg.lat_share : s->cfg.lat_share < 0 ? 0u : (unsigned)s->nctx;
  int mode = fdgpu_ed25519_get_cu_exclusive( c );            /* any mode with an exclusive walk gets its share */
  if( mode >= 1 && mode <= 3 && fdgpu_ed25519_set_lat_share( c, share ) ) goto fail;
  fdgpu_ed25519_set_record_fp_off( c, 10 );          /* offsetof( fd_txn_m_t, txn_t_sz ) */
  if( fdgpu_ed25519_prepare( c, 1 ) ) goto fail;
  if( s->launcher && fdgpu_ed25519_set_launcher( c, s->launcher ) ) goto fail;
  return c;
fail:
  fdgpu_ed25519_ctx_delete( c );
  return NULL;
}

int
fdgpu_vsvc_start( fdgpu_vsvc_t * s, int device ) {
  if( !s || !s->creator || s->started ) return -1;
  vsvc_hdr_t * h = s->h;
  s->device = device;
  s->nctx = s->cfg.nctx ? s->cfg.nctx : 2;
  if( s->nctx < 1 ) s->nctx = 1;
  if( s->nctx > VSVC_NCTX_MAX ) s->nctx = VSVC_NCTX_MAX;
  if( !s->cfg.max_wait_ns )  s->cfg.max_wait_ns  = 2000000UL;
  if( !s->cfg.copy_wait_ns ) s->cfg.copy_wait_ns = FDGPU_VTILE_COPY_WAIT_NS;
  if( !s->cfg.copy_min )     s->cfg.copy_min     = FDGPU_VTILE_COPY_MIN;
  if( !s->cfg.max_inflight ) s->cfg.max_inflight = 2UL;
  s->batch_ns = 500e3;
  s->pcap = (ulong)s->nclients * s->ring;
  s->pend    = (vsvc_pend_t *)calloc( s->pcap, sizeof(vsvc_pend_t) );
  s->p_tags  = (ulong *)malloc( s->cfg.batch_txn * sizeof(ulong) );
  s->p_dtag  = (ulong *)malloc( s->cfg.batch_txn * sizeof(ulong) );
  s->p_codes = (signed char *)malloc( s->cfg.batch_txn );
  s->p_fp    = (unsigned short *)malloc( s->cfg.batch_txn * sizeof(unsigned short) );
  int rc = -1;
  if( !s->pend || !s->p_tags || !s->p_dtag || !s->p_codes || !s->p_fp ) goto fail;
  rc = -2;
  if( s->cfg.launcher && !( s->launcher = fdgpu_launcher_new( device, s->cfg.launcher_core - 1 ) ) ) goto fail;
  for( int c=0; c<s->nclients; c++ )                         /* tiles attached before the start */
    if( atomic_load_explicit( &h->client[c].state, memory_order_acquire ) == 1 ) {
      s->seeds[c] = h->client[c].seed; s->attached[c] = 1;
    }
  for( int k=0; k<s->nctx; k++ ) if( !( s->ctx[k] = sv_ctx_new( s, k ) ) ) goto fail;
  /* the in regions: registered here unless they already lie in a registration of this process */
  rc = -3;
  for( int i=0; i<FDGPU_VSVC_RGN_MAX; i++ ) {
    if( !s->rgn_sz[i] ) continue;
    void * d = fdgpu_host_dev_ptr( s->rgn_host[i], s->rgn_sz[i] );
    if( !d ) {
      if( fdgpu_host_register( s->rgn_host[i], s->rgn_sz[i] ) ) goto fail;
      s->rgn_reg[i] = 1;
      d = fdgpu_host_dev_ptr( s->rgn_host[i], s->rgn_sz[i] );
      if( !d ) goto fail;
    }
    s->rgn_dev[i] = (uchar *)d;
  }
  /* the tiles' out dcaches: one registration over all of them */
  {
    ulong lo = s->off_out[0], hi = s->off_out[ s->nclients - 1 ] + s->out_sz;
    if( fdgpu_host_register( s->base + lo, hi - lo ) ) goto fail;
    s->out_reg = 1;
    for( int c=0; c<s->nclients; c++ ) {
      s->out_dev[c] = (uchar *)fdgpu_host_dev_ptr( s->base + s->off_out[c], s->out_sz );
      if( !s->out_dev[c] ) goto fail;
    }
  }
  s->started = 1;
  atomic_store_explicit( &h->heartbeat, sv_now(), memory_order_release );
  atomic_store_explicit( &h->ready, 1, memory_order_release );
  return 0;
fail:
  fprintf( stderr, "fdgpu_vsvc_start: %d: %s\n", rc, fdgpu_last_error() );
  atomic_store_explicit( &h->ready, -1, memory_order_release );
  return rc;
}

/* ---- the loop ----------------------------------------------------------------- */

static inline vsvc_req_t * sv_req( fdgpu_vsvc_t * s, int c ) { return (vsvc_req_t *)( s->base + s->off_req[c] ); }
static inline vsvc_cpl_t * sv_cpl( fdgpu_vsvc_t * s, int c ) { return (vsvc_cpl_t *)( s->base + s->off_cpl[c] ); }

/* launch decision (fdgpu_vtile_housekeep's, for the service's contexts): 1 if context f's filling batch
   should go now */
static int
sv_should_launch( fdgpu_vsvc_t * s, int f, ulong now, ulong * filling ) {
  ulong inflight, mi = s->cfg.max_inflight > 3UL ? 3UL : s->cfg.max_inflight;
  if( fdgpu_ed25519_faulted( s->ctx[f] ) ) return 0;
  fdgpu_ed25519_pipeline_state( s->ctx[f], filling, &inflight );
  if( !*filling || inflight >= mi ) return 0;
  if( *filling < s->cfg.min_batch && now - s->fill_t0 < s->cfg.max_wait_ns ) return 0;
  if( s->nctx > 1 && *filling < s->cfg.batch_txn ) {
    ulong stagger = (ulong)( s->batch_ns / (double)s->nctx );
    for( int k=0; k<s->nctx; k++ )
      if( k != f && s->busy[k] && now - s->launch_ns[k] < stagger ) return 0;
  }
  return 1;
}

static void
sv_launched( fdgpu_vsvc_t * s, int k, ulong now ) {
  s->launch_ns[k] = now; s->busy[k] = 1;
  ulong f, i, infl = 0UL;
  for( int j=0; j<s->nctx; j++ ) { fdgpu_ed25519_pipeline_state( s->ctx[j], &f, &i ); infl += i; }
  if( infl > s->st.gm.inflight_max ) s->st.gm.inflight_max = infl;
}

static void
sv_flush( fdgpu_vsvc_t * s ) {
  for( int i=0; i<s->nctx; i++ ) {
    int k = ( s->fill + 1 + i ) % s->nctx;              /* oldest first: the fill context's batch is the newest */
    ulong filling, inflight;
    if( fdgpu_ed25519_faulted( s->ctx[k] ) ) continue;
    fdgpu_ed25519_pipeline_state( s->ctx[k], &filling, &inflight );
    if( filling && !fdgpu_ed25519_flush( s->ctx[k] ) ) sv_launched( s, k, sv_now() );
  }
  s->copy_t0 = 0UL;
}

/* the frag at the head of the pending FIFO leaves: its completion into its tile's ring (not yet published) */
static inline void
sv_complete( fdgpu_vsvc_t * s, vsvc_pend_t const * e, int code, unsigned fp, ulong dtag, ulong bt, ulong bp, int k, int path,
             uchar * touched ) {
  int c = (int)e->client;
  vsvc_cpl_t * q = &sv_cpl( s, c )[ s->cpl_n[c] & ( s->ring - 1UL ) ];
  q->dtag = dtag; q->req = (unsigned)e->req; q->code = (short)code; q->fp = (unsigned short)fp;
  q->batch_txns = (unsigned)bt; q->batch_pos = (unsigned)bp; q->ctx = (uchar)( k < 0 ? 255 : k ); q->path = (signed char)path;
  s->cpl_n[c]++;
  touched[c] = 1;
  if( s->pcopy == s->phead ) { s->copied_n[c]++; s->pcopy++; }   /* (a verdict implies its copy completed) */
  s->phead++;
  s->st.completed++;
}

int
fdgpu_vsvc_poll( fdgpu_vsvc_t * s ) {
  if( !s->started ) return 0;
  vsvc_hdr_t * h = s->h;
  int const C = s->nclients;
  ulong t0 = sv_now(), now = t0;
  int work = 0;
  uchar touched[ FDGPU_VSVC_CLIENT_MAX ] = { 0 }, copied_ch[ FDGPU_VSVC_CLIENT_MAX ] = { 0 };
  if( now - s->t_hb > 100000UL ) { s->t_hb = now; atomic_store_explicit( &h->heartbeat, now, memory_order_release ); }
  s->st.polls++;

  /* tiles attaching (their seeds) and the test hook */
  int want_flush = 0, want_gather = 0;
  for( int c=0; c<C; c++ ) {
    vsvc_client_t * k = &h->client[c];
    if( !s->attached[c] && atomic_load_explicit( &k->state, memory_order_acquire ) == 1 ) {
      s->attached[c] = 1; s->seeds[c] = k->seed;
      for( int j=0; j<s->nctx; j++ ) if( s->ctx[j] ) fdgpu_ed25519_set_dedup_seeds( s->ctx[j], s->seeds, C );
    }
    if( !s->attached[c] ) continue;
    if( s->cfg.debug_hooks ) {                          /* (tests only: otherwise no tile can fault the contexts) */
      int f = atomic_exchange_explicit( &k->dbg_fault, 0, memory_order_acq_rel );   /* bit k: fault context k */
      for( int j=0; j<s->nctx; j++ ) if( ( f >> j ) & 1 ) fdgpu_ed25519_debug_fault( s->ctx[j] );
    }
    ulong fl = atomic_load_explicit( &k->flush, memory_order_acquire );
    if( fl != s->flush_seen[c] ) { s->flush_seen[c] = fl; want_flush = 1; }
    ulong ga = atomic_load_explicit( &k->gather, memory_order_acquire );
    if( ga != s->gather_seen[c] ) { s->gather_seen[c] = ga; want_gather = 1; }
  }

  /* intake: each tile's new requests in its order, tiles in turn (at most 256 of a tile per pass) */
  int stalled = 0;
  for( int ci=0; ci<C && !stalled; ci++ ) {
    int c = (int)( ( s->rr + (ulong)ci ) % (ulong)C );
    if( !s->attached[c] ) continue;
    vsvc_client_t * k = &h->client[c];
    ulong tail = atomic_load_explicit( &k->req_tail, memory_order_acquire );
    ulong mask = s->ring - 1UL, took = 0UL;
    vsvc_req_t const * rq = sv_req( s, c );
    while( s->next[c] < tail && took < 256UL ) {
      if( s->ptail - s->phead >= s->pcap ) { stalled = 1; break; }
      /* one read of the request: the tile can rewrite its ring at any time, so what is checked below is what is
         submitted */
      vsvc_req_t rq_local;
      memcpy( &rq_local, &rq[ s->next[c] & mask ], sizeof(vsvc_req_t) );
      __asm__ __volatile__( "" : : "r"( &rq_local ) : "memory" );
      vsvc_req_t const * r = &rq_local;
      if( s->next[c] + 2UL < tail ) __builtin_prefetch( &rq[ ( s->next[c] + 2UL ) & mask ] );
      /* a faulted context takes nothing more: the next healthy one (none: the frag completes as a fault) */
      int f = s->fill;
      for( int i=0; i<s->nctx && fdgpu_ed25519_faulted( s->ctx[f] ); i++ ) f = ( f + 1 ) % s->nctx;
      if( f != s->fill ) s->fill = f;
      vsvc_pend_t * e = &s->pend[ s->ptail % s->pcap ];
      e->client = (unsigned)c; e->req = s->next[c]; e->k = -1; e->cidx = 0UL;
      if( !fdgpu_ed25519_faulted( s->ctx[f] ) ) {
        ulong rg = r->src >> 56, off = r->src & VSVC_OFF_MASK;
        uchar const * src; uchar const * src_dev;
        /* every place a request names is checked against its region: a tile's request never makes the GPU
           read or write outside what the service registered for it */
        if( rg == VSVC_RGN_OUT && off + r->rec_sz + 16UL <= s->out_sz ) {
          src = s->base + s->off_out[c] + off; src_dev = s->out_dev[c] + off;
        }
        else if( rg < FDGPU_VSVC_RGN_MAX && s->rgn_dev[rg] && off + ( ( r->rec_sz + 15UL ) & ~15UL ) <= s->rgn_sz[rg] ) {
          src = s->rgn_host[rg] + off; src_dev = s->rgn_dev[rg] + off;
        } else src = src_dev = NULL;
        ulong const * seq_dev = NULL;
        if( r->line != VSVC_LINE_NONE ) {
          ulong lr = r->line >> 56, lo = r->line & VSVC_OFF_MASK;
          if( lr < FDGPU_VSVC_RGN_MAX && s->rgn_dev[lr] && lo + 8UL <= s->rgn_sz[lr] ) seq_dev = (ulong const *)( s->rgn_dev[lr] + lo );
          else src = NULL;
        }
        ulong dsto = (ulong)r->dst_chunk * FDGPU_CHUNK_SZ;
        int rc = -1;
        if( src && r->rec_sz >= FDGPU_TXNM_HDR_SZ && r->rec_sz <= FDGPU_TXNM_HDR_SZ + 1232UL &&
            dsto + SV_RESERVE_MAX <= s->out_sz ) {
          unsigned flags = FDGPU_GATHER_SEED( c ) | ( ( r->flags & VSVC_REQ_HOSTCOPY ) ? FDGPU_GATHER_NO_WRITEBACK : 0U );
          rc = fdgpu_ed25519_submit_raw_gather_to( s->ctx[f], src, src_dev, s->out_dev[c] + dsto, r->rec_sz,
                                                   (unsigned short)FDGPU_TXNM_HDR_SZ,
                                                   (unsigned short)( r->rec_sz - FDGPU_TXNM_HDR_SZ ), s->ptail, seq_dev,
                                                   r->seq, flags );
        }
        if( rc == -2 ) { stalled = 1; break; }                 /* every staging slot in flight: drain first */
        if( !rc ) {
          e->k = f; e->cidx = s->sub_cnt[f]++;
          ulong fl, in; fdgpu_ed25519_pipeline_state( s->ctx[f], &fl, &in );
          if( fl == 1UL ) s->fill_t0 = now;
          if( !s->copy_t0 ) s->copy_t0 = now;
        } else if( rc != -3 ) {
          /* a request the service cannot place (outside its regions): refused -- completes as a fault */
          fprintf( stderr, "fdgpu_vsvc: tile %d request %lu refused (%d): %s\n", c, s->next[c], rc, fdgpu_last_error() );
        }
      }
      s->ptail++; s->next[c]++; took++;
      s->st.taken++;
    }
    if( took ) { atomic_store_explicit( &k->taken, s->next[c], memory_order_relaxed ); work = 1; }
  }
  s->rr++;

  /* launches (adaptive, as a tile's housekeep), early copies */
  now = sv_now();
  for( int k=0; k<s->nctx; k++ ) {                        /* batch duration: a context's batches have drained */
    if( !s->busy[k] ) continue;
    ulong f, i; fdgpu_ed25519_pipeline_state( s->ctx[k], &f, &i );
    if( !i ) { s->busy[k] = 0; s->batch_ns = 0.875*s->batch_ns + 0.125*(double)( now - s->launch_ns[k] ); }
  }
  if( want_flush ) { sv_flush( s ); work = 1; }
  else {
    ulong filling;
    int f = s->fill;
    if( sv_should_launch( s, f, now, &filling ) ) {
      if( !fdgpu_ed25519_flush( s->ctx[f] ) ) {
        sv_launched( s, f, now ); s->fill = ( f + 1 ) % s->nctx; s->copy_t0 = 0UL; work = 1;
      }
    } else if( ( want_gather || ( s->copy_t0 && ( now - s->copy_t0 >= s->cfg.copy_wait_ns ||
                                                  s->sub_cnt[f] - fdgpu_ed25519_gather_launched( s->ctx[f] ) >= s->cfg.copy_min ) ) )
               && !fdgpu_ed25519_faulted( s->ctx[f] ) ) {
      if( fdgpu_ed25519_gather( s->ctx[f] ) > 0 ) { s->st.gm.copies++; work = 1; }
      s->copy_t0 = 0UL;
    }
    if( want_gather )
      for( int k=0; k<s->nctx; k++ ) if( k != f && !fdgpu_ed25519_faulted( s->ctx[k] ) ) (void)fdgpu_ed25519_gather( s->ctx[k] );
  }

  /* copy progress: the tiles' copied prefixes (what their reliable links' credits wait for) */
  ulong g[ VSVC_NCTX_MAX ];
  for( int k=0; k<s->nctx; k++ ) g[k] = fdgpu_ed25519_gathered( s->ctx[k] );
  if( s->pcopy < s->phead ) s->pcopy = s->phead;
  while( s->pcopy < s->ptail ) {
    vsvc_pend_t const * e = &s->pend[ s->pcopy % s->pcap ];
    if( e->k < 0 || e->cidx >= g[ e->k ] ) break;
    s->copied_n[ e->client ]++; copied_ch[ e->client ] = 1;
    s->pcopy++;
  }

  /* verdicts, in the order taken: the run of pending frags at the head that went to one context is its oldest
     launched batch */
  while( s->phead < s->ptail ) {
    vsvc_pend_t const * e = &s->pend[ s->phead % s->pcap ];
    int k = e->k;
    if( k < 0 || fdgpu_ed25519_faulted( s->ctx[k] ) ) {
      if( k >= 0 && !s->fault_seen[k] ) { s->fault_seen[k] = 1; s->st.faults++; }
      sv_complete( s, e, VSVC_CODE_FAULT, 0U, 0UL, 0UL, 0UL, k, FDGPU_PATH_NONE, touched );
      s->st.fault_completions++; work = 1;
      continue;
    }
    ulong want = fdgpu_ed25519_front_remaining( s->ctx[k] );
    if( !want ) break;
    if( want > s->cfg.batch_txn ) want = s->cfg.batch_txn;
    ulong bt, bc; int bp;
    fdgpu_ed25519_front_batch( s->ctx[k], &bt, &bc, &bp );
    ulong got = fdgpu_ed25519_poll_raw( s->ctx[k], s->p_tags, s->p_codes, NULL, s->p_fp, s->p_dtag, want, 0 );
    if( !got ) break;                                      /* (faulted just now: completed on the next pass) */
    if( !bc ) {                                            /* a batch's first verdicts: did it hold several tiles' frags? */
      unsigned c0 = e->client;
      for( ulong i=1; i<bt && s->phead + i < s->ptail; i++ )
        if( s->pend[ ( s->phead + i ) % s->pcap ].client != c0 ) { s->st.mixed_batches++; break; }
    }
    for( ulong i=0; i<got; i++ ) {
      e = &s->pend[ s->phead % s->pcap ];
      if( s->p_tags[i] != s->phead ) {
        fprintf( stderr, "fdgpu_vsvc_poll: completion tag %lu != pending frag %lu\n", s->p_tags[i], s->phead );
        abort();
      }
      sv_complete( s, e, (int)s->p_codes[i], s->p_fp[i], s->p_dtag[i], bt, bc + i, k, bp, touched );
    }
    work = 1;
  }
  for( int c=0; c<C; c++ ) {
    if( touched[c] ) atomic_store_explicit( &h->client[c].cpl_tail, s->cpl_n[c], memory_order_release );
    if( touched[c] || copied_ch[c] ) atomic_store_explicit( &h->client[c].copied, s->copied_n[c], memory_order_release );
  }

  /* faulted contexts: recreated once none of the pending frags is theirs */
  int nf = 0;
  for( int k=0; k<s->nctx; k++ ) {
    if( !fdgpu_ed25519_faulted( s->ctx[k] ) ) continue;
    int busy = 0;
    for( ulong q=s->phead; q<s->ptail && !busy; q++ ) busy = s->pend[ q % s->pcap ].k == k;
    fdgpu_ed25519_ctx_t * nc = busy ? NULL : sv_ctx_new( s, k );
    if( nc ) {
      fdgpu_ed25519_ctx_delete( s->ctx[k] ); s->ctx[k] = nc;
      s->busy[k] = 0; s->fault_seen[k] = 0; s->sub_cnt[k] = 0UL; s->st.recovered++;
    } else nf++;
  }
  atomic_store_explicit( &h->faulted, nf, memory_order_relaxed );

  ulong dt = sv_now() - t0;
  s->st.loop_ns += dt;
  if( work ) { s->st.busy_polls++; s->st.busy_ns += dt; }
  return work;
}

int
fdgpu_vsvc_run( fdgpu_vsvc_t * s ) {
  while( !atomic_load_explicit( &s->h->stop, memory_order_acquire ) )
    if( !fdgpu_vsvc_poll( s ) ) _mm_pause();
  return 0;
}

void
fdgpu_vsvc_stats( fdgpu_vsvc_t * s, fdgpu_vsvc_stats_t * out ) {
  *out = s->st;
  fdgpu_vtile_gpu_metrics_t * gm = &out->gm;
  memset( gm->lat_hist, 0, sizeof(gm->lat_hist) );
  memset( gm->gather_gpu, 0, sizeof(gm->gather_gpu) );
  memset( gm->phase, 0, sizeof(gm->phase) );
  gm->batches = gm->batch_txns = gm->launch_ns = 0UL;
  ulong infl = 0UL;
  for( int k=0; k<s->nctx; k++ ) {
    if( !s->ctx[k] ) continue;
    ulong f, i; fdgpu_ed25519_pipeline_state( s->ctx[k], &f, &i ); infl += i;
    ulong b, t, hh[ FDGPU_LAT_BUCKETS ];
    fdgpu_ed25519_batch_stats( s->ctx[k], &b, &t, hh );
    gm->batches += b; gm->batch_txns += t;
    for( int j=0; j<FDGPU_LAT_BUCKETS; j++ ) gm->lat_hist[j] += hh[j];
    ulong lns, nl; fdgpu_ed25519_launch_stats( s->ctx[k], &lns, &nl ); gm->launch_ns += lns;
    ulong gs[8]; fdgpu_ed25519_gather_stats( s->ctx[k], gs );
    for( int j=0; j<8; j++ ) {
      if( j == 2 || j == 4 || j == 6 ) { if( gs[j] > gm->gather_gpu[j] ) gm->gather_gpu[j] = gs[j]; }
      else gm->gather_gpu[j] += gs[j];
    }
    ulong ph[9]; fdgpu_ed25519_phase_stats( s->ctx[k], ph );
    for( int j=0; j<9; j++ ) {
      if( j == 2 || j == 4 || j == 6 ) { if( ph[j] > gm->phase[j] ) gm->phase[j] = ph[j]; }
      else gm->phase[j] += ph[j];
    }
  }
  if( s->launcher ) fdgpu_launcher_stats( s->launcher, gm->launcher );
  else memset( gm->launcher, 0, sizeof(gm->launcher) );
  gm->inflight = infl;
  gm->pending = s->ptail - s->phead;
  gm->faults = s->st.faults;
  gm->gpu_fault_frags = s->st.fault_completions;
}

void
fdgpu_vsvc_delete( fdgpu_vsvc_t * s ) {
  if( !s ) return;
  for( int k=0; k<VSVC_NCTX_MAX; k++ ) if( s->ctx[k] ) fdgpu_ed25519_ctx_delete( s->ctx[k] );
  fdgpu_launcher_delete( s->launcher );
  for( int i=0; i<FDGPU_VSVC_RGN_MAX; i++ ) if( s->rgn_reg[i] ) fdgpu_host_unregister( s->rgn_host[i] );
  if( s->out_reg ) fdgpu_host_unregister( s->base + s->off_out[0] );
  free( s->pend ); free( s->p_tags ); free( s->p_dtag ); free( s->p_codes ); free( s->p_fp );
  if( s->creator && s->path[0] ) unlink( s->path );
  munmap( s->base, s->sz );
  free( s );
}

/* Test hook (no GPU call): a CPU stand-in for the service's GPU side, so the rings and a served tile's logic
   are checked on a machine without a GPU (tests/test_vsvc.py).  Takes every request published so far and
   completes it at once: the record is copied from its place into the tile's out dcache (as the GPU's copy
   writes it back) with txn_t_sz = fp, after the overrun check the GPU makes (a changed in-mcache line:
   FDGPU_ERR_OVERRUN); the code is codes[ request index % ncodes ]; the HA dedup tag is XXH64( tile seed,
   payload bytes 1..64 ) (a one-signature transaction's signature).  Only on a service not started.  Returns
   the requests completed. */
ulong
fdgpu_vsvc_debug_serve( fdgpu_vsvc_t * s, int const * codes, ulong ncodes, ulong fp ) {
  if( !s || !s->creator || s->started || !codes || !ncodes ) return 0UL;
  vsvc_hdr_t * h = s->h;
  ulong done = 0UL;
  for( int c=0; c<s->nclients; c++ ) {
    vsvc_client_t * k = &h->client[c];
    if( !s->attached[c] ) {
      if( atomic_load_explicit( &k->state, memory_order_acquire ) != 1 ) continue;
      s->attached[c] = 1; s->seeds[c] = k->seed;
    }
    ulong tail = atomic_load_explicit( &k->req_tail, memory_order_acquire ), mask = s->ring - 1UL;
    vsvc_req_t const * rq = sv_req( s, c );
    vsvc_cpl_t * cq = sv_cpl( s, c );
    uchar * out = s->base + s->off_out[c];
    for( ; s->next[c] < tail; s->next[c]++, done++ ) {
      vsvc_req_t rq_local;
      memcpy( &rq_local, &rq[ s->next[c] & mask ], sizeof(vsvc_req_t) );
      __asm__ __volatile__( "" : : "r"( &rq_local ) : "memory" );
      vsvc_req_t const * r = &rq_local;
      ulong rg = r->src >> 56, off = r->src & VSVC_OFF_MASK;
      uchar const * src = rg == VSVC_RGN_OUT ? ( off + r->rec_sz <= s->out_sz ? out + off : NULL )
                        : rg < FDGPU_VSVC_RGN_MAX && s->rgn_host[rg] && off + r->rec_sz <= s->rgn_sz[rg] ? s->rgn_host[rg] + off : NULL;
      if( (ulong)r->dst_chunk * FDGPU_CHUNK_SZ + r->rec_sz > s->out_sz ) src = NULL;
      uchar * dst = out + (ulong)r->dst_chunk * FDGPU_CHUNK_SZ;
      int code = codes[ s->next[c] % ncodes ];
      ulong dtag = 0UL;
      if( !src ) code = VSVC_CODE_FAULT;
      else {
        if( !( r->flags & VSVC_REQ_HOSTCOPY ) && src != dst ) memmove( dst, src, r->rec_sz );
        if( r->line != VSVC_LINE_NONE ) {
          ulong lr = r->line >> 56, lo = r->line & VSVC_OFF_MASK;
          ulong const * w = lr < FDGPU_VSVC_RGN_MAX && s->rgn_host[lr] && lo + 8UL <= s->rgn_sz[lr]
                          ? (ulong const *)( s->rgn_host[lr] + lo ) : NULL;
          if( !w || atomic_load_explicit( (_Atomic ulong const *)w, memory_order_acquire ) != r->seq ) code = FDGPU_ERR_OVERRUN;
        }
        if( code != FDGPU_ERR_OVERRUN ) {
          *(unsigned short *)( dst + 10 ) = (unsigned short)fp;
          if( r->rec_sz >= FDGPU_TXNM_HDR_SZ + 65UL ) dtag = fdgpu_dedup_tag( s->seeds[c], dst + FDGPU_TXNM_HDR_SZ + 1 );
        }
      }
      vsvc_cpl_t * q = &cq[ s->cpl_n[c] & mask ];
      q->dtag = dtag; q->req = (unsigned)s->next[c]; q->code = (short)code; q->fp = code == FDGPU_ERR_OVERRUN ? 0 : (unsigned short)fp;
      q->batch_txns = 0U; q->batch_pos = 0U; q->ctx = 0; q->path = (signed char)FDGPU_PATH_NONE;
      s->cpl_n[c]++; s->copied_n[c]++;
    }
    atomic_store_explicit( &k->taken, s->next[c], memory_order_relaxed );
    atomic_store_explicit( &k->copied, s->copied_n[c], memory_order_release );
    atomic_store_explicit( &k->cpl_tail, s->cpl_n[c], memory_order_release );
  }
  atomic_store_explicit( &h->heartbeat, sv_now(), memory_order_release );
  atomic_store_explicit( &h->ready, 1, memory_order_release );   /* (the tiles' liveness check: serving) */
  return done;
}
