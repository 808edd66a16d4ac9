#ifndef HEADER_ref_stem_h
#define HEADER_ref_stem_h
/* ref_stem.h -- TEST INFRASTRUCTURE ONLY: the run configuration of
   ref_stem_harness.c (oracle/_ref/libfdref_stem.so), mirrored by
   oracle/oracle.py _StemCfg (layout checked by tests/test_ref_stem.py). */

typedef struct {
  /* inputs */
  unsigned char const * payload;    /* payload p at payload + off[p], sz[p] bytes (<= 1232) */
  unsigned int const *  off;
  unsigned short const * sz;
  unsigned long n_payload;
  unsigned long n_frags;                    /* the producer's frag s carries payload s % n_payload */
  unsigned long in_depth;                   /* in mcache depth (power of 2) */
  unsigned long out_depth;                  /* out mcache depth */
  unsigned long batch_txn, tcache_depth, seed;
  unsigned long rate_fps;                   /* producer pace (0: unthrottled) */
  unsigned long consumer_pause_every;       /* the consumer sleeps consumer_pause_ns every this many frags (0: never) */
  unsigned long consumer_pause_ns;
  unsigned long max_inflight;
  int   device, nctx, zero_copy;
  int   _pad;
  /* outputs */
  unsigned long * tr_seq; int * tr_res; unsigned long * tr_tag; unsigned long tr_cap;           /* the tile's verdicts */
  unsigned long * c_seq_in; unsigned long * c_hash; unsigned long * c_sz; unsigned long c_cap;         /* what the consumer received, in order */
  unsigned long out[ 16 ];  /* verdicts, consumed, returned, stem_overruns(marked), filtered, taken, published, bursts,
                       metric: in consumed, in filtered, in overrun polling, in overrun reading, backpressure count,
                       tile metrics[0..1] (parse, verify fails) */
  unsigned long tile_metrics[ 5 ];
} ref_stem_cfg_t;

int ref_stem_run( ref_stem_cfg_t * c );

#endif
