#ifndef HEADER_fd_vsvc_private_h
#define HEADER_fd_vsvc_private_h

/* fd_vsvc_private.h -- the verify service's shared segment (include/fd_verify_gpu.h, fdgpu_vsvc_*), as
   both sides see it: the service process (fd_vsvc.c) and the tile processes it serves
   (fd_verify_gpu.c, fdgpu_vtile_new_svc).

   Segment: this header; then per client (verify tile) a request ring, a completion ring (ring_cap
   entries each, ring_cap >= the frags a tile can have pending) and the tile's out dcache (2 MiB
   aligned).  Every ring is single-producer / single-consumer: the tile writes requests and publishes
   req_tail (release), the service reads them; the service writes completions and publishes cpl_tail
   (release), the tile reads them.  Neither side waits for the other's consumption: a tile never has
   more than ring_cap frags between during_frag and after_frags. */

#include "../../include/fd_verify_gpu.h"
#include <stdatomic.h>

#define VSVC_MAGIC        (0xfd75c0de00000006UL)
#define VSVC_OFF_MASK     ((1UL << 56) - 1UL)
#define VSVC_RGN_OUT      (255UL)   /* a request's source is the tile's own out dcache (a record the tile copied) */
#define VSVC_LINE_NONE    (~0UL)    /* no overrun check for the request */
#define VSVC_CODE_FAULT   (-128)    /* the frag's GPU batch failed: no verdict (FDGPU_VTILE_GPU_FAULT) */
#define VSVC_REQ_HOSTCOPY (1U)      /* the record is already in place in the out dcache: the GPU reads it, no write-back */

typedef struct {                    /* tile -> service, one per frag, in the tile's during_frag order: 32 bytes */
  unsigned long  seq;               /* the frag's seq on its in link (for the overrun check) */
  unsigned long  src;               /* region id << 56 | byte offset of the record (fd_txn_m_t) in it */
  unsigned long  line;              /* region id << 56 | byte offset of its in-mcache line's seq word, or VSVC_LINE_NONE */
  unsigned int   dst_chunk;         /* the record's chunk in the tile's out dcache */
  unsigned short rec_sz;            /* header + payload bytes */
  unsigned short flags;             /* VSVC_REQ_* */
} vsvc_req_t;

typedef struct {                    /* service -> tile, one per request, in request order: 32 bytes */
  unsigned long  dtag;              /* HA dedup tag (the tile's seed) */
  unsigned int   req;               /* low 32 bits of the request's index (checked by the tile) */
  short          code;              /* FD_ED25519_*, FDGPU_ERR_PARSE / _OVERRUN, or VSVC_CODE_FAULT */
  unsigned short fp;                /* fd_txn_t footprint (0: not parsed) */
  unsigned int   batch_txns, batch_pos;   /* the GPU batch (diagnostics, fdgpu_vtile_done_t) */
  unsigned char  ctx;               /* the service's engine context */
  signed char    path;              /* FDGPU_PATH_* or latency lanes */
  unsigned char  _pad[ 6 ];
} vsvc_cpl_t;

typedef struct __attribute__(( aligned( 64 ) )) {
  /* written by the tile */
  _Atomic unsigned long req_tail;   /* requests published */
  _Atomic unsigned long flush;      /* bumped: launch the filling batches now (fdgpu_vtile_flush, a blocking drain) */
  _Atomic unsigned long gather;     /* bumped: start the copies of every frag taken (fdgpu_vtile_copy) */
  _Atomic int           state;      /* 0 free, 1 attached, 2 detached */
  _Atomic int           dbg_fault;  /* test hook: bit k = fault the service's engine context k (fdgpu_vtile_debug_fault) */
  unsigned long         seed;       /* the tile's HA dedup seed (written before state = 1) */
  long                  pid;
  unsigned char         _pad0[ 8 ];
  /* written by the service */
  _Atomic unsigned long cpl_tail __attribute__(( aligned( 64 ) ));   /* completions published */
  _Atomic unsigned long copied;     /* the tile's first `copied` requests have been copied by the GPU (or completed) */
  _Atomic unsigned long taken;      /* requests the service has taken */
  /* layout (written at creation) */
  unsigned long         off_req __attribute__(( aligned( 64 ) ));
  unsigned long         off_cpl, off_out, ring_cap, out_sz;
} vsvc_client_t;

typedef struct {
  _Atomic unsigned long magic;      /* set last by the creator (release) */
  unsigned long         total_sz;
  int                   clients;
  int                   _pad;
  unsigned long         ring_cap, out_sz;
  _Atomic unsigned long heartbeat;  /* the service loop's clock (ns), refreshed every ~100 us while it polls */
  _Atomic int           ready;      /* 1 started, -1 its start failed */
  _Atomic int           stop;
  _Atomic int           faulted;    /* the service's engine contexts faulted now */
  int                   _pad1;
  _Atomic unsigned long joined;
  unsigned long         rgn_sz[ FDGPU_VSVC_RGN_MAX ];   /* the regions the service added (0: none) */
  vsvc_client_t         client[ FDGPU_VSVC_CLIENT_MAX ];
} vsvc_hdr_t;

#define VSVC_NCTX_MAX 3

typedef struct {                    /* the service's pending frag (all tiles, in the order taken) */
  unsigned int  client;
  int           k;                  /* engine context (-1: refused, completes as a fault) */
  unsigned long req;                /* the tile's request index */
  unsigned long cidx;               /* its index among context k's gathered submissions */
} vsvc_pend_t;

struct fdgpu_vsvc {
  vsvc_hdr_t *          h;
  unsigned char *       base;
  unsigned long         sz;
  int                   creator;    /* made the segment (file: unlinks it at delete) */
  char                  path[ 256 ];
  /* the creator's private copy of the layout: the service never takes a size or an offset from the
     segment, which every tile can write */
  int                   nclients;
  unsigned long         ring, out_sz;
  unsigned long         off_req[ FDGPU_VSVC_CLIENT_MAX ], off_cpl[ FDGPU_VSVC_CLIENT_MAX ], off_out[ FDGPU_VSVC_CLIENT_MAX ];
  /* service side (fdgpu_vsvc_start) */
  fdgpu_vsvc_cfg_t      cfg;
  int                   started, device, nctx;
  fdgpu_ed25519_ctx_t * ctx[ VSVC_NCTX_MAX ];
  fdgpu_launcher_t *    launcher;
  unsigned char *       rgn_host[ FDGPU_VSVC_RGN_MAX ];
  unsigned char *       rgn_dev[ FDGPU_VSVC_RGN_MAX ];
  unsigned long         rgn_sz[ FDGPU_VSVC_RGN_MAX ];
  int                   rgn_reg[ FDGPU_VSVC_RGN_MAX ];
  unsigned char *       out_dev[ FDGPU_VSVC_CLIENT_MAX ];
  int                   out_reg;
  unsigned long         seeds[ FDGPU_VSVC_CLIENT_MAX ];
  int                   attached[ FDGPU_VSVC_CLIENT_MAX ];
  unsigned long         next[ FDGPU_VSVC_CLIENT_MAX ];      /* requests taken per client */
  unsigned long         cpl_n[ FDGPU_VSVC_CLIENT_MAX ];     /* completions written per client */
  unsigned long         copied_n[ FDGPU_VSVC_CLIENT_MAX ];  /* copied prefix per client */
  unsigned long         flush_seen[ FDGPU_VSVC_CLIENT_MAX ], gather_seen[ FDGPU_VSVC_CLIENT_MAX ];
  vsvc_pend_t *         pend;
  unsigned long         pcap, phead, ptail, pcopy;
  unsigned long         sub_cnt[ VSVC_NCTX_MAX ];
  int                   fill, busy[ VSVC_NCTX_MAX ], fault_seen[ VSVC_NCTX_MAX ];
  unsigned long         launch_ns[ VSVC_NCTX_MAX ];
  double                batch_ns;
  unsigned long         fill_t0, copy_t0, t_hb, rr;
  unsigned long         *p_tags, *p_dtag;
  signed char *         p_codes;
  unsigned short *      p_fp;
  fdgpu_vsvc_stats_t    st;
};

/* a tile concludes the service is gone when its heartbeat is older than this (its blocking waits then end
   with every pending frag as FDGPU_VTILE_GPU_FAULT) */
#define VSVC_DEAD_NS (3000000000UL)

#endif /* HEADER_fd_vsvc_private_h */
