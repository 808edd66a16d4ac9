#ifndef HEADER_fd_ed25519_gpu_h
#define HEADER_fd_ed25519_gpu_h

/* fd_ed25519_gpu.h -- C ABI of the MI355X batch ed25519 verify engine
   (libfdgpu_ed25519.so).

   Two layers:

   1. Drop-in synchronous API.  Same names, signatures, argument meaning
      and result codes as the reference's ballet/ed25519 verify API, so
      a caller such as fd_verify_tile links this library in place of
      the ballet ed25519 verify objects without source changes:

        fd_ed25519_verify                  <- src/ballet/ed25519/fd_ed25519.h:96-101
                                              (impl fd_ed25519_user.c:135-230)
        fd_ed25519_verify_batch_single_msg <- src/ballet/ed25519/fd_ed25519.h:124-130
                                              (impl fd_ed25519_user.c:232-310)
        fd_ed25519_strerror                <- src/ballet/ed25519/fd_ed25519.h:137-138
                                              (impl fd_ed25519_user.c:312-322)
        FD_ED25519_SUCCESS/ERR_SIG/ERR_PUBKEY/ERR_MSG
                                           <- src/ballet/ed25519/fd_ed25519.h:11-14

      The fd_sha512_t * arguments are accepted and ignored (the GPU
      computes SHA-512 itself); they are kept so the prototypes are
      identical.  These calls each run one GPU round trip, so they are
      correct but latency-bound; throughput comes from layer 2.  Any
      message length is accepted, as in the reference: when 96*batch_sz +
      msg_sz passes the 16-bit descriptor range (every verify-path message
      is <= 1232 bytes) the digests SHA-512(R||A||M) are computed by the
      batch SHA-512 kernel first and handed to the verify kernels.  Codes
      are always FD_ED25519_*; a GPU runtime failure aborts the process
      (the reference has no such failure mode; a verify tile's failure
      is an FD_LOG_ERR, fd_verify_tile.c:74-84).

   2. Batch / async API (new; prefix fdgpu_).  A batch is a set of
      transactions described by fdgpu_txn_desc_t records (the fields
      fd_txn_verify reads from fd_txn_t, src/disco/verify/
      fd_verify_tile.h:59-108) over a byte arena of payloads.  Each
      transaction's signature_cnt signatures are verified over its
      message with fd_ed25519_verify_batch_single_msg semantics.

   All pointers are plain C pointers; "d_" prefixed arguments are HIP
   device pointers, "stream" is a hipStream_t passed as void *.
   No torch / C++ types cross this boundary. */

#ifdef __cplusplus
extern "C" {
#endif

#ifndef FD_ED25519_SUCCESS
#define FD_ED25519_SUCCESS    ( 0) /* Operation was successful */
#define FD_ED25519_ERR_SIG    (-1) /* signature was obviously invalid */
#define FD_ED25519_ERR_PUBKEY (-2) /* public key was obviously invalid */
#define FD_ED25519_ERR_MSG    (-3) /* message didn't match the signature */
#endif

#ifndef HEADER_fd_src_ballet_sha512_fd_sha512_h
/* Opaque in this ABI; same tag as src/ballet/sha512/fd_sha512.h:129 so
   the prototypes below are compatible with the reference header. */
typedef struct fd_sha512_private fd_sha512_t;
#endif

/* ---- Layer 1: drop-in synchronous API ----------------------------- */

int
fd_ed25519_verify( unsigned char const   msg[], /* msg_sz */
                   unsigned long         msg_sz,
                   unsigned char const   sig[ 64 ],
                   unsigned char const   public_key[ 32 ],
                   fd_sha512_t *         sha );

int
fd_ed25519_verify_batch_single_msg( unsigned char const   msg[], /* msg_sz */
                                    unsigned long const   msg_sz,
                                    unsigned char const   signatures[ 64 ], /* 64 * batch_sz */
                                    unsigned char const   pubkeys[ 32 ],    /* 32 * batch_sz */
                                    fd_sha512_t *         shas[ 1 ],        /* batch_sz */
                                    unsigned char const   batch_sz );

char const *
fd_ed25519_strerror( int err );

/* ---- Layer 2: batch / async API ------------------------------------ */

/* Result-code semantics.  The reference's AVX-512 (r43x6) and portable
   (ref) backends agree on accept/reject but differ in two codes
   (SURVEY.md §0.2): a public key that fails to decode gives ERR_SIG on
   AVX-512 and ERR_PUBKEY on ref, and an encoding with x==0 and the
   sign bit set is rejected at decode by AVX-512 only.  AVX-512 is the
   default (it is the north-star CPU baseline). */
#define FDGPU_ERR_TOO_LONG     (-4)   /* submit: the record cannot fit the ctx payload arena (not queued) */

#define FDGPU_SEMANTICS_AVX512 (0)
#define FDGPU_SEMANTICS_REF    (1)

#define FDGPU_TXN_MTU          (1232UL) /* FD_TPU_MTU, src/disco/fd_txn_m_t.h */
#define FDGPU_SIG_MAX          (16UL)   /* fd_ed25519_user.c:238 MAX */

/* One transaction of a batch.  16 bytes.  payload_off is the byte
   offset of the payload in the batch arena; sig_base is the index of
   this transaction's first signature in the per-signature output
   (the exclusive prefix sum of sig_cnt, computed by the stager).
   signature_off / acct_addr_off / message_off are the fd_txn_t fields
   of the same name (src/ballet/txn/fd_txn.h); message bytes are
   [message_off, payload_sz).  A transaction with sig_cnt==0 or
   sig_cnt>16 gets FD_ED25519_ERR_SIG, exactly like
   fd_ed25519_verify_batch_single_msg (fd_ed25519_user.c:238-241). */
typedef struct fdgpu_txn_desc {
  unsigned int   payload_off;
  unsigned int   sig_base;
  unsigned short payload_sz;
  unsigned short message_off;
  unsigned short acct_addr_off;
  unsigned char  signature_off;
  unsigned char  sig_cnt;
} fdgpu_txn_desc_t;

/* Raw-payload batches (the verify tile's after_frag work, fd_txn_parse +
   fd_txn_verify, src/disco/verify/fd_verify_tile.c:110-140, moved onto
   the GPU).  One 16-byte record per transaction: the stager only copies
   the payload and reads its first byte.  sig_lanes = payload[0] if
   1 <= payload[0] <= 16, else 0 (a parsed transaction's signature_cnt
   is its first byte, fd_txn_parse.c:86); sig_base = exclusive prefix
   sum of sig_lanes.  The device parses every payload
   (fd_txn_parse_core semantics), derives the fdgpu_txn_desc_t itself and
   verifies the parsed transactions.  Per-transaction result:
   FDGPU_ERR_PARSE if fd_txn_parse rejects the payload, else the
   fd_ed25519_verify_batch_single_msg code (ERR_SIG for signature_cnt
   > 16). */
typedef struct fdgpu_txn_raw {
  unsigned int   payload_off;
  unsigned int   sig_base;
  unsigned short payload_sz;
  unsigned char  sig_lanes;
  unsigned char  _pad[ 5 ];
} fdgpu_txn_raw_t;

#define FDGPU_ERR_PARSE        (-16)    /* fd_txn_parse returned 0 */
#define FDGPU_ERR_OVERRUN      (-17)    /* gathered record: its in-mcache line was reused while the GPU copied it
                                           (fdgpu_ed25519_submit_raw_gather_chk); never parsed or verified */
#define FDGPU_TXN_IMG_STRIDE   (864UL)  /* >= FD_TXN_MAX_SZ (852), fd_txn.h:99 */

/* A context is single-threaded (one per verify tile / thread); several
   contexts may share a device.  If a batch fails on the device, poll
   stops at it, fdgpu_last_error says why and every later submit returns
   -3: delete and recreate the context. */
typedef struct fdgpu_ed25519_ctx fdgpu_ed25519_ctx_t;

/* fdgpu_ed25519_ctx_new creates an engine bound to HIP device `device`
   sized for batches of up to max_txn transactions / max_sig signatures
   / max_payload_bytes of payload arena.  Allocates device scratch and
   pinned staging buffers (call before entering a seccomp sandbox, i.e.
   from privileged_init).  Returns NULL on failure (see
   fdgpu_last_error). */
fdgpu_ed25519_ctx_t *
fdgpu_ed25519_ctx_new( int           device,
                       unsigned long max_txn,
                       unsigned long max_sig,
                       unsigned long max_payload_bytes,
                       int           semantics );

void
fdgpu_ed25519_ctx_delete( fdgpu_ed25519_ctx_t * ctx );

/* fdgpu_ed25519_verify_txns_device enqueues verification of a batch
   whose arena and descriptors are already resident in device memory.
   Writes one code per transaction to d_txn_out[txn_cnt] and one code
   per signature to d_sig_out[sig_cnt] (the code fd_ed25519_verify
   would return for that signature alone; may be NULL).  Asynchronous
   on `stream` (NULL = the ctx's own stream).  Returns 0 on successful
   enqueue, negative on bad arguments. */
int
fdgpu_ed25519_verify_txns_device( fdgpu_ed25519_ctx_t *    ctx,
                                  unsigned char const *    d_payload,
                                  fdgpu_txn_desc_t const * d_desc,
                                  unsigned long            txn_cnt,
                                  unsigned long            sig_cnt,
                                  signed char *            d_txn_out,
                                  signed char *            d_sig_out,
                                  void *                   stream );

/* fdgpu_ed25519_verify_txns_host: same from host memory; stages through
   the ctx's pinned buffers, runs, and waits.  Synchronous.  A payload
   that lies inside one fdgpu_host_alloc / fdgpu_host_register-ed region
   (a pinned dcache) is DMA'd to the device directly, with no staging
   copy. */
int
fdgpu_ed25519_verify_txns_host( fdgpu_ed25519_ctx_t *    ctx,
                                unsigned char const *    payload,
                                unsigned long            payload_bytes,
                                fdgpu_txn_desc_t const * desc,
                                unsigned long            txn_cnt,
                                signed char *            txn_out,
                                signed char *            sig_out );

/* fdgpu_txn_parse_device: batch fd_txn_parse (src/ballet/txn/fd_txn.h:
   713-715 / fd_txn_parse.c:6-252) on the device.  Transaction t is
   d_payload[ d_raw[t].payload_off, +payload_sz ); its fd_txn_t image
   goes to d_img + t*img_stride (img_stride >= 852; d_img may be NULL)
   and its footprint (0 = rejected) to d_fp[t].  Only payload_off and
   payload_sz of d_raw are read.  Asynchronous on `stream`. */
int
fdgpu_txn_parse_device( unsigned char const *   d_payload,
                        fdgpu_txn_raw_t const * d_raw,
                        unsigned long           txn_cnt,
                        unsigned char *         d_img,
                        unsigned long           img_stride,
                        unsigned short *        d_fp,
                        void *                  stream );

/* fdgpu_ed25519_verify_raw_device: parse + verify a raw-payload batch
   resident in device memory (see fdgpu_txn_raw_t).  sig_cnt = sum of
   sig_lanes.  d_txn_out[t] gets FDGPU_ERR_PARSE or the batch verify
   code; d_img / d_fp (optional) get the parser's fd_txn_t images and
   footprints, which the tile publishes after the payload
   (fd_verify_tile.c:111).  Asynchronous. */
int
fdgpu_ed25519_verify_raw_device( fdgpu_ed25519_ctx_t *   ctx,
                                 unsigned char const *   d_payload,
                                 fdgpu_txn_raw_t const * d_raw,
                                 unsigned long           txn_cnt,
                                 unsigned long           sig_cnt,
                                 signed char *           d_txn_out,
                                 unsigned char *         d_img,
                                 unsigned long           img_stride,
                                 unsigned short *        d_fp,
                                 void *                  stream );

/* fdgpu_ed25519_verify_raw_host: the same from host memory (payload
   arena + raw records; sig_lanes / sig_base are recomputed here from
   the payloads, so only payload_off / payload_sz need be set).
   Synchronous.  img (txn_cnt*img_stride bytes) and fp may be NULL. */
int
fdgpu_ed25519_verify_raw_host( fdgpu_ed25519_ctx_t *   ctx,
                               unsigned char const *   payload,
                               unsigned long           payload_bytes,
                               fdgpu_txn_raw_t *       raw,
                               unsigned long           txn_cnt,
                               signed char *           txn_out,
                               unsigned char *         img,
                               unsigned long           img_stride,
                               unsigned short *        fp );

/* fdgpu_ed25519_verify_many_host: out[i] = fd_ed25519_verify( msgs[i],
   msg_szs[i], sigs[i], pubs[i] ) for cnt independent triples, in GPU
   batches of up to max_txn (the batched form of fd_ed25519_verify for the
   gossip / precompile callers).  Synchronous; needs a ctx
   with staging (max_payload_bytes > 0); messages up to 65439 bytes. */
int
fdgpu_ed25519_verify_many_host( fdgpu_ed25519_ctx_t *         ctx,
                                unsigned char const * const * msgs,
                                unsigned long const *         msg_szs,
                                unsigned char const * const * sigs,
                                unsigned char const * const * pubs,
                                unsigned long                 cnt,
                                signed char *                 out );

/* fdgpu_ed25519_verify_txn_ptrs: out[i] = the fd_ed25519_verify_batch_
   single_msg code of transaction i, whose payload is at payloads[i] (any
   host memory) and whose fd_txn_t fields are in desc[i] (signature_off,
   acct_addr_off, message_off, sig_cnt, payload_sz; payload_off and
   sig_base ignored).  The replay path's batched fd_executor_txn_verify
   (src/flamenco/runtime/fd_executor.c:1550-1574): one call per block
   instead of one CPU verify per transaction.  Synchronous; needs a ctx
   with staging. */
int
fdgpu_ed25519_verify_txn_ptrs( fdgpu_ed25519_ctx_t *         ctx,
                               unsigned char const * const * payloads,
                               fdgpu_txn_desc_t const *      desc,
                               unsigned long                 cnt,
                               signed char *                 out );

/* Batch SHA-512 (replaces fd_sha512_batch_init / add / fini,
   src/ballet/sha512/fd_sha512.h:234-419, for any number of messages):
   hash[64 t, 64 t + 64) = SHA-512 of the sz[t] bytes at data + off[t].
   The device form reads up to 132 bytes past each message's last whole
   128-byte block, so d_data must carry 256 readable bytes of slack after
   its last message.  The host form copies, runs on `device` and waits. */
int
fdgpu_sha512_batch_device( unsigned char const * d_data,
                           unsigned long const * d_off,
                           unsigned int const *  d_sz,
                           unsigned long         cnt,
                           unsigned char *       d_hash,
                           void *                stream );

int
fdgpu_sha512_batch_host( int                   device,
                         unsigned char const * data,
                         unsigned long         data_sz,
                         unsigned long const * off,
                         unsigned int const *  sz,
                         unsigned long         cnt,
                         unsigned char *       hash );

/* Async submit / poll pipeline (the offload shape fd_verify_tile needs,
   SURVEY.md §8b).  submit copies one transaction payload into the
   current pinned staging slot; when the slot fills (or on flush) it is
   launched (H2D copy + kernels + D2H copy on the ctx stream) and the
   next slot becomes current.  poll returns completed verdicts in
   submission order: out_tags[i] is the tag given to submit and
   out_codes[i] the fd_ed25519_verify_batch_single_msg code.  Returns
   the number written (<= max).  submit returns 0 on success, -1 if
   the transaction is malformed (it is then completed with ERR_SIG),
   -2 if all slots are in flight (caller should poll), -3 if the ctx has
   faulted, FDGPU_ERR_TOO_LONG if the record (payload_sz + 8 bytes)
   exceeds max_payload_bytes (nothing is queued). */
int
fdgpu_ed25519_submit( fdgpu_ed25519_ctx_t * ctx,
                      unsigned char const * payload,
                      unsigned short        payload_sz,
                      unsigned char         signature_off,
                      unsigned short        acct_addr_off,
                      unsigned short        message_off,
                      unsigned char         sig_cnt,
                      unsigned long         tag );

int
fdgpu_ed25519_flush( fdgpu_ed25519_ctx_t * ctx );

/* Batch latency histogram buckets (async pipeline: slot launch -> the
   verdicts seen by poll): bucket 0 < 32 us, bucket i in 1..38 covers
   [32 us * 2^((i-1)/4), 32 us * 2^(i/4)) (quarter octaves up to ~23 ms),
   bucket 39 the rest. */
#define FDGPU_LAT_BUCKETS (40)
static inline int fdgpu_lat_bucket( unsigned long ns ) {
  if( ns < 32000UL ) return 0;
  int oct = 63 - __builtin_clzl( ns / 32000UL );            /* ns / 32 us in [2^oct, 2^(oct+1)) */
  unsigned long base = 32000UL << oct;
  int quarter = ( ns*10000UL >= base*11892UL ) + ( ns*10000UL >= base*14142UL ) + ( ns*10000UL >= base*16818UL );
  int b = 1 + 4*oct + quarter;
  return b < FDGPU_LAT_BUCKETS - 1 ? b : FDGPU_LAT_BUCKETS - 1;
}
/* counters of ctx's async pipeline: batches launched, transactions in them,
   and (hist, may be NULL) the latency histogram above */
void
fdgpu_ed25519_batch_stats( fdgpu_ed25519_ctx_t const * ctx, unsigned long * batches, unsigned long * txns,
                           unsigned long hist[ FDGPU_LAT_BUCKETS ] );

/* host time the caller's thread spent inside ctx's batch launches (the
   HIP calls that queue a batch's copies and kernels), ns, and how many */
void
fdgpu_ed25519_launch_stats( fdgpu_ed25519_ctx_t const * ctx, unsigned long * launch_ns, unsigned long * launches );

/* Launch thread (no reference counterpart: the reference's verify tile makes no runtime calls).  A
   launcher is a thread, pinned to `cpu` (-1: not pinned), that makes the HIP runtime calls of the
   async batches and copies of the contexts attached to it, in the order they were queued, so the
   caller's thread spends a queue push per batch instead of the calls themselves (~40 us per latency-path
   batch).  Polls are unchanged.  A failed call faults its context.  fdgpu_ed25519_set_launcher (L NULL:
   detach) needs a context with nothing pending; a context is deleted before its launcher.  Commands are
   queued by one thread at a time: the contexts of one launcher belong to one caller thread (a verify
   tile).  Stats: commands issued, ns spent issuing them, the deepest queue seen, pushes that waited for
   room, the longest single command (ns: a runtime call that blocked) and how many took over 250 us. */
typedef struct fdgpu_launcher fdgpu_launcher_t;
fdgpu_launcher_t * fdgpu_launcher_new( int device, int cpu );
void               fdgpu_launcher_delete( fdgpu_launcher_t * launcher );
void               fdgpu_launcher_stats( fdgpu_launcher_t const * launcher, unsigned long out[ 6 ] );
int                fdgpu_ed25519_set_launcher( fdgpu_ed25519_ctx_t * ctx, fdgpu_launcher_t * launcher );

/* 1 once a batch of ctx has failed on the device (poll then returns 0
   without blocking and every submit returns -3: the in-flight
   transactions are lost; delete and recreate the ctx). */
int
fdgpu_ed25519_faulted( fdgpu_ed25519_ctx_t const * ctx );

/* Test hook (host side only): ctx behaves from now on exactly as after a
   failed batch. */
void
fdgpu_ed25519_debug_fault( fdgpu_ed25519_ctx_t * ctx );
/* Test hook: with on, ctx's launch thread (fdgpu_ed25519_set_launcher) fails every batch launch it makes
   from now on, as a failed runtime call would -- the context faults asynchronously, on that thread. */
void
fdgpu_ed25519_debug_fail_launch( fdgpu_ed25519_ctx_t * ctx, int on );

/* Signatures of the last batch launched on ctx that took the full 253-bit
   walk instead of the half-size one (no short (c0, c1) pair, or forced by
   fdgpu_debug_opts_t.half_force_slow); 0 when the half-size path is off.
   TEST-ONLY: it synchronises ctx's stream (stalling any async batch in
   flight) and sees only the last batch launched, so it is not a metric a
   tile loop can export.  A device reduction that silently failed would
   still verify correctly, only slower. */
unsigned long
fdgpu_ed25519_slow_count( fdgpu_ed25519_ctx_t * ctx );

unsigned long
fdgpu_ed25519_poll( fdgpu_ed25519_ctx_t * ctx,
                    unsigned long *       out_tags,
                    signed char *         out_codes,
                    unsigned long         max,
                    int                   blocking );

/* transactions of ctx's oldest launched batch not yet returned by a poll
   (0 if none is in flight): the most one poll can return without moving
   on to the next batch */
unsigned long
fdgpu_ed25519_front_remaining( fdgpu_ed25519_ctx_t const * ctx );

/* Engine path a batch ran (diagnostics): the latency path's lanes per signature in the walk (8, 4, 2, 1),
   the throughput path's half-size walk, its full-length walk, or a batch with no signatures */
#define FDGPU_PATH_THROUGHPUT       (0)
#define FDGPU_PATH_THROUGHPUT_FULL  (-1)
#define FDGPU_PATH_NONE             (-2)
/* ctx's oldest launched batch: its transactions, how many a poll has returned, and its FDGPU_PATH_* (or
   lanes); 0 if none is in flight */
int
fdgpu_ed25519_front_batch( fdgpu_ed25519_ctx_t const * ctx, unsigned long * txn_cnt, unsigned long * cursor,
                           int * path );

/* Pipeline occupancy: transactions in the slot being filled, and
   launched slots not yet fully drained by poll.  Lets a caller launch
   early when the GPU is idle and let batches grow while it is busy. */
void
fdgpu_ed25519_pipeline_state( fdgpu_ed25519_ctx_t const * ctx,
                              unsigned long *             filling,
                              unsigned long *             inflight );

/* Raw-payload form of the pipeline (what fd_verify_tile's during_frag /
   after_frag pair needs, with fd_txn_parse moved onto the GPU):
   submit_raw copies one raw payload (no host parse); poll_raw returns,
   in submission order, the tag, the code (FDGPU_ERR_PARSE or the batch
   verify code), and, when out_img / out_fp are non-NULL, the parser's
   fd_txn_t image (out_img + i*FDGPU_TXN_IMG_STRIDE, footprint bytes) and
   footprint.  A slot holds one kind of submission; switching kinds
   flushes.  Returns as fdgpu_ed25519_submit / fdgpu_ed25519_poll. */
int
fdgpu_ed25519_submit_raw( fdgpu_ed25519_ctx_t * ctx,
                          unsigned char const * payload,
                          unsigned short        payload_sz,
                          unsigned long         tag );

/* In-place form (zero-copy staging): the payload already sits at
   `payload` inside a pinned region starting at `base` (the tile's out
   dcache, allocated with fdgpu_host_alloc); a batch uploads the
   contiguous range of its payloads straight from the region instead of
   a staging copy.  Payloads of one batch must lie at increasing addresses
   of one region (a lower address, e.g. a ring wrap, starts a new batch)
   with 512 readable bytes after each; the caller keeps them unchanged
   until poll_raw returns their verdicts.  Completions come back through
   fdgpu_ed25519_poll_raw. */
int
fdgpu_ed25519_submit_raw_ref( fdgpu_ed25519_ctx_t * ctx,
                              unsigned char const * base,
                              unsigned char const * payload,
                              unsigned short        payload_sz,
                              unsigned long         tag );

/* pinned (page-locked) host memory for fdgpu_ed25519_submit_raw_ref regions */
void * fdgpu_host_alloc( unsigned long sz );
void   fdgpu_host_free ( void * p );

/* Page-lock an existing host range and map it for the GPU (a tile's in
   dcache: the workspace the producer writes frags into), so that
   fdgpu_ed25519_submit_raw_gather can read records there.  0 on
   success; -2 if a registered range already starts at p.
   fdgpu_host_register_shared: for holders sharing one range (verify
   tiles' handles on one mcache ring): the first registers it, each later
   call with exactly the same (p, sz) takes another reference, and the
   range stays mapped until as many fdgpu_host_unregister( p ) calls.  1
   (nothing taken) if that range was registered by fdgpu_host_register
   (its owner keeps it mapped); -2 for another size at p. */
int    fdgpu_host_register       ( void * p, unsigned long sz );
int    fdgpu_host_register_shared( void * p, unsigned long sz );
void   fdgpu_host_unregister     ( void * p );

/* NUMA node of HIP device `device` (its PCI function's numa_node in
   sysfs), -1 if unknown: where the threads that drive it and their pinned
   buffers belong. */
int    fdgpu_device_numa_node( int device );

/* Gathered form (no host copy at all; the zero-copy staging of SURVEY.md
   §8f rank 2): the record -- copy_sz bytes at src, 16-B aligned, inside
   a range given to fdgpu_host_register or fdgpu_host_alloc, with the
   transaction payload at src + payload_off -- stays where the producer
   wrote it.  The batch's first kernel reads it over PCIe, into the
   device arena and into dst: the record's place in the caller's pinned
   out region dst_base (from fdgpu_host_alloc).  So after poll_raw
   returns its verdict the out region holds the record, as if the host
   had copied it (the reference's during_frag copy, fd_verify_tile.c:
   77-79).  Records of one batch lie at increasing dst addresses of one
   region (a lower one starts a new batch), 16-B aligned, with room for
   copy_sz rounded up to 16 at dst; src must stay valid until the record's
   gather has completed (fdgpu_ed25519_gathered; at the latest, its
   verdict).  The GPU also writes each parsed transaction's fd_txn_t image into the out
   region, behind the payload at the next 2-byte boundary (where the
   tile publishes it), so poll_raw returns footprints but leaves out_img
   untouched for these transactions; leave room for 852 bytes there. */
int
fdgpu_ed25519_submit_raw_gather( fdgpu_ed25519_ctx_t * ctx,
                                 unsigned char const * src,
                                 unsigned char *       dst_base,
                                 unsigned char *       dst,
                                 unsigned short        copy_sz,
                                 unsigned short        payload_off,
                                 unsigned short        payload_sz,
                                 unsigned long         tag );

/* The same with the stem's overrun check (src/disco/stem/fd_stem.c:667-686)
   done by the GPU: seq_addr (NULL = no check; else 8-B aligned, inside a
   registered range) is the seq word of the frag's line in the producer's
   mcache, and seq the value it held when the caller took the frag.  Right
   after copying the record the gather kernel re-reads that word (a
   system-scope load behind every copy load); if it changed, the producer
   reused the line while the record was being read, and the record's
   verdict is FDGPU_ERR_OVERRUN.  The decision is made once, at copy time:
   a lap after the gather has completed changes nothing. */
int
fdgpu_ed25519_submit_raw_gather_chk( fdgpu_ed25519_ctx_t * ctx,
                                     unsigned char const * src,
                                     unsigned char *       dst_base,
                                     unsigned char *       dst,
                                     unsigned short        copy_sz,
                                     unsigned short        payload_off,
                                     unsigned short        payload_sz,
                                     unsigned long         tag,
                                     unsigned long const * seq_addr,
                                     unsigned long         seq );

/* Early gather: launch now, on the context's gather stream, the copies of
   every gathered record submitted to the filling batch and not yet
   copied (the batch itself launches later; its kernels wait for these
   copies).  This is what bounds how long a frag stays exposed to the
   producer between during_frag and its copy.  Returns the number of
   records launched (0: none pending), < 0 on error.
   fdgpu_ed25519_gathered: records (all gathered submissions of ctx, in
   submission order, counted from 0) whose copy has completed -- read from
   a pinned word the last block of each gather stores; no HIP call.
   fdgpu_ed25519_gather_launched: records whose copy has been launched. */
long          fdgpu_ed25519_gather( fdgpu_ed25519_ctx_t * ctx );
unsigned long fdgpu_ed25519_gathered( fdgpu_ed25519_ctx_t const * ctx );
unsigned long fdgpu_ed25519_gather_launched( fdgpu_ed25519_ctx_t const * ctx );
/* Reserve n CUs for ctx's gathers: its verify kernels run on the other
   CUs (a CU-masked stream) and the gathers on those n only, so a copy
   starts at once however busy the verify kernels keep the GPU (without
   a reservation a gather waits for wave slots the verify kernels hold).
   Only on a fresh context (before any submit).  0, or < 0 (e.g. the
   runtime refused CU masks: the context is unchanged). */
int           fdgpu_ed25519_reserve_gather_cus( fdgpu_ed25519_ctx_t * ctx, unsigned n );
/* The same, with the verify kernels confined to the part-th of `parts`
   equal shares of the CUs the gathers leave (reserve_gather_cus = part 0
   of 1): the contexts of one tile, given parts 0..parts-1, never place
   their concurrent batches' waves on the same SIMDs. */
int           fdgpu_ed25519_reserve_cus( fdgpu_ed25519_ctx_t * ctx, unsigned n, unsigned part, unsigned parts );
/* gathers timed on the GPU clock (mapped to host time once): out[0] how
   many, out[1] / out[2] the sum / max of host launch -> first block's
   start, out[3] / out[4] the sum / max of first block's start -> last
   block's end, out[5] / out[6] the sum / max of the runtime call that
   issued it (on the launch thread, if any: after its queue) -> first
   block's start, ns, out[7] how many of those took over 250 us */
void          fdgpu_ed25519_gather_stats( fdgpu_ed25519_ctx_t * ctx, unsigned long out[ 8 ] );
/* where the async batches' time goes, from GPU clock stamps at each batch's
   verify kernels' start and end (mapped to host time once, at context
   creation): out[0] batches timed; out[1] / out[2] sum / max of host launch
   -> its verify kernels start (waiting for its gathers and for the stream's
   earlier batch); out[3] / out[4] sum / max of kernels start -> end;
   out[5] / out[6] sum / max of end -> poll saw it; out[7] / out[8] sum and
   count of launch -> its last gather ended (gathered batches), ns */
void          fdgpu_ed25519_phase_stats( fdgpu_ed25519_ctx_t const * ctx, unsigned long out[ 9 ] );
/* make now every allocation the async pipeline otherwise makes on first use (all staging slots; raw:
   the raw-payload buffers and the gather stream too), so that batches later make no allocation
   syscalls -- a tile calls it in privileged init, before its sandbox.  0, or < 0 */
int           fdgpu_ed25519_prepare( fdgpu_ed25519_ctx_t * ctx, int raw );
/* fdgpu_ed25519_submit_raw_gather_chk with the device views of src and of the seq word given by the
   caller (translated once per registered region, fdgpu_host_region), so the per-frag call does no
   region lookup.  Same checks and results. */
int           fdgpu_ed25519_submit_raw_gather_dev( fdgpu_ed25519_ctx_t * ctx, unsigned char const * src,
                                                   unsigned char const * src_dev, unsigned char * dst_base,
                                                   unsigned char * dst, unsigned short copy_sz, unsigned short payload_off,
                                                   unsigned short payload_sz, unsigned long tag,
                                                   unsigned long const * seq_dev, unsigned long seq );
/* ... with flags: FDGPU_GATHER_NO_WRITEBACK -- the GPU copies the record into its arena (and re-checks the
   seq) but does not write it back to dst: the caller copies bytes [0, 10) and [12, copy_sz) of the record
   there itself (host copy threads, fdgpu_vtile_opts_t.copy_threads), the GPU still writes the record's
   txn_t_sz (bytes 10-11, with fdgpu_ed25519_set_record_fp_off 10) and its fd_txn_t image.  The record then
   crosses PCIe once (read) instead of twice. */
#define FDGPU_GATHER_NO_WRITEBACK (1U)
int           fdgpu_ed25519_submit_raw_gather_dev_f( fdgpu_ed25519_ctx_t * ctx, unsigned char const * src,
                                                     unsigned char const * src_dev, unsigned char * dst_base,
                                                     unsigned char * dst, unsigned short copy_sz,
                                                     unsigned short payload_off, unsigned short payload_sz,
                                                     unsigned long tag, unsigned long const * seq_dev,
                                                     unsigned long seq, unsigned flags );
/* Per-record form (the verify service, fdgpu_vsvc_*: one batch takes the frags of several verify tiles,
   and each record goes back into its own tile's out dcache): as fdgpu_ed25519_submit_raw_gather_dev_f, but
   the record's place on the host is given by its device address dst_dev alone (16-B aligned, inside a
   registered range, room for copy_sz rounded up to 16 plus 852 bytes of fd_txn_t image), with no order
   between the records of a batch.  The batch arena takes records in submission order.  A batch holds
   records of one form: switching forms launches the filling batch.  Same results.  flags may also carry
   FDGPU_GATHER_SEED( i ): the record's HA dedup tag is computed with seed i of
   fdgpu_ed25519_set_dedup_seeds (each verify tile has a secure seed of its own, fd_verify_tile.c:166). */
#define FDGPU_GATHER_SEED( i ) ( ( (unsigned)(i) & 15u ) << 8 )
/* n (0..16) per-record HA dedup seeds (0: back to the single seed of fdgpu_ed25519_set_dedup); turns the
   dedup tags on.  0, or -1 */
int           fdgpu_ed25519_set_dedup_seeds( fdgpu_ed25519_ctx_t * ctx, unsigned long const * seeds, int n );
int           fdgpu_ed25519_submit_raw_gather_to( fdgpu_ed25519_ctx_t * ctx, unsigned char const * src,
                                                  unsigned char const * src_dev, unsigned char * dst_dev,
                                                  unsigned short copy_sz, unsigned short payload_off,
                                                  unsigned short payload_sz, unsigned long tag,
                                                  unsigned long const * seq_dev, unsigned long seq, unsigned flags );
/* the region registered with fdgpu_host_register / fdgpu_host_alloc that holds p: its host base, size and
   device base; 0, or -1 if p is in none */
int           fdgpu_host_region( void const * p, void ** base, unsigned long * sz, void ** dev_base );
/* wait until every launched gather of ctx has completed: 0, or -3 (ctx faulted) */
int           fdgpu_ed25519_gather_wait( fdgpu_ed25519_ctx_t * ctx );

/* device address of the host range [p, p+sz) if it lies inside one range
   given to fdgpu_host_register / fdgpu_host_alloc, else NULL */
void * fdgpu_host_dev_ptr( void const * p, unsigned long sz );

/* out_dedup (may be NULL): with fdgpu_ed25519_set_dedup on, the HA dedup
   tag of each parsed transaction (XXH64 of its first signature with the
   set seed, exactly fd_txn_verify's fd_hash( seed, sig0, 64 ),
   fd_verify_tile.h:79; 0 for a rejected payload), computed on the GPU so
   the tile never reads the payload bytes on the host. */
unsigned long
fdgpu_ed25519_poll_raw( fdgpu_ed25519_ctx_t * ctx,
                        unsigned long *       out_tags,
                        signed char *         out_codes,
                        unsigned char *       out_img,
                        unsigned short *      out_fp,
                        unsigned long *       out_dedup,
                        unsigned long         max,
                        int                   blocking );

void
fdgpu_ed25519_set_dedup( fdgpu_ed25519_ctx_t * ctx, int enable, unsigned long seed );

/* Gathered records (fdgpu_ed25519_submit_raw_gather) whose header holds a
   u16 footprint field at byte `off` (fd_txn_m_t txn_t_sz: 10): the GPU
   stores each footprint there as well, next to the fd_txn_t image, so
   the tile never writes the record either.  -1 (default) = none.  Needs
   payload_off <= 255 and off + 2 <= payload_off in every gathered
   record. */
int
fdgpu_ed25519_set_record_fp_off( fdgpu_ed25519_ctx_t * ctx, int off );

/* Batches of at most small_max signatures take the latency path: one
   launch decodes A, decodes R and hashes side by side, and R is compared
   at the end of the DSM.  Larger batches take the throughput path: R is
   not decompressed up front but checked against P's encoding after one
   batched inversion per 256 signatures.  Both give identical codes.
   Default FD_SMALL_BATCH_MAX (fdgpu_debug_set_opts can change the value
   new contexts start with); 0 forces the throughput path, ~0UL the
   latency path.
   Returns the previous value. */
unsigned long
fdgpu_ed25519_set_small_batch_max( fdgpu_ed25519_ctx_t * ctx, unsigned long small_max );

/* 1: every workgroup of the latency path's prep and walk kernels reserves
   more than half of a CU's LDS (unused), so each runs alone on its CU --
   two contexts' concurrent small batches then never share a SIMD (a
   tile's staggered contexts, fdgpu_vtile_opts_t.cu_exclusive).  0: off
   (default).  A/B variants: 2 = at most two per CU, 3 = the walk only,
   4 = the prep only.  The throughput path is never affected.  0 or < 0. */
int
fdgpu_ed25519_set_cu_exclusive( fdgpu_ed25519_ctx_t * ctx, int on );
/* ctx's mode: 0 off (the default), 1..4 as set, -1 off as chosen by fdgpu_debug_opts_t.cu_exclusive (a
   verify tile then does not apply its own default, fdgpu_vtile_opts_t.cu_exclusive) */
int
fdgpu_ed25519_get_cu_exclusive( fdgpu_ed25519_ctx_t const * ctx );

/* ctx's share of the CUs for its exclusive latency-path walk: with n > 0
   the walk counts on (CUs - ctx's reserved gather CUs) / n of them; 0 (the
   default): no limit.  With cu_exclusive on, a walk of more workgroups
   than CUs free waits for CUs to drain, and the dispatcher holding its
   tail holds the kernels queued behind it -- another context's walk,
   gathers -- so a backlog grows batches and feeds itself.  Within a
   share the latency path takes the most lanes per signature (8, 4, 2, 1)
   whose walk fits: a tile with n contexts gives each 1/n.  After
   fdgpu_ed25519_reserve_cus.  0 on success, -1 bad ctx, -2 HIP error. */
int
fdgpu_ed25519_set_lat_share( fdgpu_ed25519_ctx_t * ctx, unsigned parts );

/* Per-kernel timing, in milliseconds: the mean over the batches launched
   since fdgpu_ed25519_set_timing(ctx,1) (at most the last 64) of HIP
   events recorded on the stream the kernels ran on.  idx: 0 = prep
   (SHA-512 + decode + checks + A-table), 1 = dsm (double-scalar
   multiplication + compare), 2 = reduce; on the throughput path the prep
   split in two: 3 = the decode kernel (A and R, the -A / -R tables), 4 =
   the hash kernel (SHA-512, k mod l, the half-size scalars).  Valid once
   those batches completed; -1 when nothing was timed. */
void
fdgpu_ed25519_set_timing( fdgpu_ed25519_ctx_t * ctx, int enable );

float
fdgpu_ed25519_kernel_ms( fdgpu_ed25519_ctx_t * ctx, int idx );

/* Diagnostics: sustained v_mad_u64_u32 rate of `device` in 32x32+64
   multiply-accumulates per second (a register-only probe kernel over the
   whole chip).  The VALU-integer roofline the kernels are priced
   against; MI355X_MICROARCH.md has no integer-multiply row. */
double
fdgpu_mad_peak_per_s( int device );

/* The drop-ins (fd_ed25519_verify, fd_ed25519_verify_batch_single_msg)
   share one process-wide context, created on first use on device 0 with
   FDGPU_SEMANTICS_AVX512.  Call this first to choose another device or
   the portable codes (recreates the context if one exists).  0 on
   success. */
int
fdgpu_ed25519_dropin_init( int device, int semantics );

/* ---- test / A/B hooks (never read from the environment) ---------------
   Options for engine contexts created after the call, process-wide
   (contexts that already exist keep theirs).  NULL restores the
   defaults.  The tests run every engine path through these; the product
   never calls it. */
typedef struct fdgpu_debug_opts {
  int           half;             /* -1: default (half-size walk); 0: full-length walk + deferred R check; 1: half */
  unsigned int  half_force_slow;  /* 0: off; m: signatures with S % m == 0 take the full-length walk (slow list) */
  long          small_batch_max;  /* -1: default; else the initial fdgpu_ed25519_set_small_batch_max */
  int           dsm_lanes;        /* latency path: lanes per signature in the DSM (1, 2, 4, 8); 0 = by batch size */
  long          nofold_max;       /* -1: default; batches of at most this many signatures use the unfolded DSM */
  int           gather_no_writeback; /* gathered records' write-back into the caller's out region: 0 = by the
                                        gather kernel as it copies (default); 2 = by the batch's fd_finish_kernel
                                        from the device arena (A/B: measured slower, profiles/r03/stream_defer);
                                        1 = DIAGNOSTIC, none (published records lack their payload) */
  int           poll_prefetch;       /* completions polled: software prefetch this many entries ahead in the
                                        GPU-written result arrays (0: none, A/B) */
  int           gather_rpb;          /* records per workgroup of the gather kernel: 0 = default (4), 1 = one (A/B) */
  int           gather_cu_spread;    /* the CUs a tile context reserves for its gathers: 0 = the last n (default),
                                        1 = every (CUs/n)-th, 2 = the first n (A/B) */
  int           cu_exclusive;        /* 1..4: new contexts start with fdgpu_ed25519_set_cu_exclusive( ctx, n ); -1: off,
                                        also in verify tiles (whose default is on); 0: default */
  int           quad_sha;            /* latency path (half-size): 0 = default, the prep's hash role on a quad of lanes per
                                        signature up to 8,192 signatures (fd_sha512_RAM_quad); -1 = one lane (A/B) */
} fdgpu_debug_opts_t;

void
fdgpu_debug_set_opts( fdgpu_debug_opts_t const * opts );

/* Diagnostics: the GPU pauses seen by this process's gather timing -- up to n of the first 512 timed gathers
   (any context) that waited over 250 us on the GPU after the runtime call that issued them, as pairs (host
   CLOCK_MONOTONIC ns of the call, ns waited) in out[2 n].  Returns how many there were (all, not only those
   copied); reset 1 starts a new log. */
unsigned long
fdgpu_debug_gather_pauses( unsigned long * out, unsigned long n, int reset );

/* Last error string of the calling thread (never NULL). */
char const *
fdgpu_last_error( void );

#ifdef __cplusplus
}
#endif

#endif /* HEADER_fd_ed25519_gpu_h */
