/* ref_harness.c -- TEST INFRASTRUCTURE ONLY.

   Thin driver compiled together with the reference's own ed25519 /
   sha512 sources (taken in place from /root/reference by
   oracle/Makefile, never copied) into oracle/_ref/libfdref_*.so.  It
   exposes the reference verify path to the Python tests / fixture
   generator / bench cpu_baseline through plain C entry points. */

#include "ballet/ed25519/fd_ed25519.h"
#include "../include/fd_ed25519_gpu.h"
#include <pthread.h>
#include <string.h>

int
ref_verify( uchar const * msg, ulong msg_sz, uchar const * sig, uchar const * pub ) {
  fd_sha512_t sha[1];
  return fd_ed25519_verify( msg, msg_sz, sig, pub, sha );
}

int
ref_verify_batch( uchar const * msg, ulong msg_sz, uchar const * sigs, uchar const * pubs, uchar n ) {
  fd_sha512_t sha_mem[ 16 ];
  fd_sha512_t * shas[ 16 ];
  for( int i=0; i<16; i++ ) shas[i] = &sha_mem[i];
  return fd_ed25519_verify_batch_single_msg( msg, msg_sz, sigs, pubs, shas, n );
}

void
ref_sign( uchar * sig, uchar const * msg, ulong msg_sz, uchar const * pub, uchar const * prv ) {
  fd_sha512_t sha[1];
  fd_ed25519_sign( sig, msg, msg_sz, pub, prv, sha );
}

void
ref_public_from_private( uchar * pub, uchar const * prv ) {
  fd_sha512_t sha[1];
  fd_ed25519_public_from_private( pub, prv, sha );
}

void
ref_sha512( uchar const * in, ulong sz, uchar * out ) {
  fd_sha512_t sha[1];
  fd_sha512_fini( fd_sha512_append( fd_sha512_init( sha ), in, sz ), out );
}

/* Batch driver with the layout of include/fd_ed25519_gpu.h.  txn code =
   fd_ed25519_verify_batch_single_msg exactly as fd_txn_verify calls it
   (src/disco/verify/fd_verify_tile.h:59-92); per-signature codes (if
   sig_out; NULL for the timed CPU baseline, which then verifies each
   signature once) = fd_ed25519_verify of each signature alone. */

typedef struct {
  uchar const * payload; fdgpu_txn_desc_t const * desc; ulong lo, hi;
  schar * txn_out; schar * sig_out;
} job_t;

static void *
job_run( void * _j ) {
  job_t * j = (job_t *)_j;
  fd_sha512_t sha_mem[ 16 ];
  fd_sha512_t * shas[ 16 ];
  for( int i=0; i<16; i++ ) shas[i] = &sha_mem[i];
  for( ulong i=j->lo; i<j->hi; i++ ) {
    fdgpu_txn_desc_t const * d = j->desc + i;
    uchar const * base = j->payload + d->payload_off;
    uint n = d->sig_cnt;
    int ok = n>=1 && n<=16
          && (uint)d->signature_off + 64u*n <= d->payload_sz
          && (uint)d->acct_addr_off + 32u*n <= d->payload_sz
          && d->message_off <= d->payload_sz;
    if( !ok ) {
      j->txn_out[i] = FD_ED25519_ERR_SIG;
      if( j->sig_out ) for( uint s=0; s<n; s++ ) j->sig_out[ d->sig_base + s ] = FD_ED25519_ERR_SIG;
      continue;
    }
    uchar const * msg = base + d->message_off;
    ulong msg_sz = (ulong)d->payload_sz - d->message_off;
    j->txn_out[i] = (schar)fd_ed25519_verify_batch_single_msg( msg, msg_sz, base + d->signature_off,
                                                               base + d->acct_addr_off, shas, (uchar)n );
    if( j->sig_out ) for( uint s=0; s<n; s++ )
      j->sig_out[ d->sig_base + s ] = (schar)fd_ed25519_verify( msg, msg_sz, base + d->signature_off + 64*s,
                                                               base + d->acct_addr_off + 32*s, shas[0] );
  }
  return NULL;
}

void
ref_verify_txns( uchar const * payload, fdgpu_txn_desc_t const * desc, ulong txn_cnt,
                 schar * txn_out, schar * sig_out, int threads ) {
  if( threads<1 ) threads = 1;
  if( threads>256 ) threads = 256;
  pthread_t th[ 256 ]; job_t jobs[ 256 ];
  for( int t=0; t<threads; t++ ) {
    jobs[t] = (job_t){ payload, desc, txn_cnt*(ulong)t/(ulong)threads, txn_cnt*(ulong)(t+1)/(ulong)threads, txn_out, sig_out };
    if( t ) pthread_create( &th[t], NULL, job_run, &jobs[t] );
  }
  job_run( &jobs[0] );
  for( int t=1; t<threads; t++ ) pthread_join( th[t], NULL );
}
