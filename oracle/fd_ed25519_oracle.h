#ifndef HEADER_fd_ed25519_oracle_h
#define HEADER_fd_ed25519_oracle_h

/* TEST INFRASTRUCTURE ONLY.  The oracle is a from-scratch CPU
   restatement of the reference's ed25519 verify path used as the parity
   checker by tests/, __graft_entry__.smoke() and bench.py's
   cpu_baseline leg.  Nothing in firedancer_amd/ links or calls it.

   Parity pinned against the compiled reference (oracle/_ref, built from
   /root/reference sources by oracle/Makefile) through the fixtures in
   tests/golden/ (CCTV, Wycheproof, malleability, fuzz corpus, edge
   encodings, seeded random cases), see tests/golden/gen_golden.py. */

#include <stddef.h>
#include <stdint.h>
#include "../include/fd_ed25519_gpu.h"

#ifdef __cplusplus
extern "C" {
#endif

void oracle_sha512( uint8_t const * in, size_t sz, uint8_t out[ 64 ] );

/* out = in mod l, in is 64 bytes little endian */
void oracle_scalar_reduce( uint8_t out[ 32 ], uint8_t const in[ 64 ] );

/* 1 if s < l (canonical), 0 otherwise */
int oracle_scalar_validate( uint8_t const s[ 32 ] );

/* Decode a point.  Returns 0 on success, 1 if not on the curve (non
   square), 2 if x==0 with sign bit set (only reported when semantics is
   FDGPU_SEMANTICS_AVX512).  On success writes canonical affine x,y. */
int oracle_point_decode( uint8_t x[ 32 ], uint8_t y[ 32 ], uint8_t const enc[ 32 ], int semantics );

int oracle_ed25519_verify( uint8_t const * msg, size_t msg_sz,
                           uint8_t const sig[ 64 ], uint8_t const pub[ 32 ],
                           int semantics );

int oracle_ed25519_verify_batch_single_msg( uint8_t const * msg, size_t msg_sz,
                                            uint8_t const * sigs, uint8_t const * pubs,
                                            uint8_t batch_sz, int semantics );

/* Verify a whole batch (same layout as the GPU batch API).  sig_out may
   be NULL.  threads<=1 runs on the calling thread. */
void oracle_verify_txns( uint8_t const * payload, fdgpu_txn_desc_t const * desc, size_t txn_cnt,
                         int8_t * txn_out, int8_t * sig_out, int semantics, int threads );

/* Test-data helpers (RFC 8032 5.1.5 / 5.1.6). */
void oracle_ed25519_public_from_private( uint8_t pub[ 32 ], uint8_t const prv[ 32 ] );
void oracle_ed25519_sign( uint8_t sig[ 64 ], uint8_t const * msg, size_t msg_sz,
                          uint8_t const pub[ 32 ], uint8_t const prv[ 32 ] );

/* [k](-A) + [S]B encoded (for kernel-level tests).  Returns 0 / -1 if A
   fails to decode. */
int oracle_dsm_encode( uint8_t out[ 32 ], uint8_t const k[ 32 ], uint8_t const A[ 32 ], uint8_t const S[ 32 ] );

#ifdef __cplusplus
}
#endif

#endif
