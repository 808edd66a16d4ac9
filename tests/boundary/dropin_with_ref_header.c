/* Compile-only check of the drop-in boundary (tests/test_boundary.py): the reference's own ed25519 header
   (src/ballet/ed25519/fd_ed25519.h, included in place from /root/reference) and then this engine's
   include/fd_ed25519_gpu.h in one translation unit, under -Wall -Werror.  Both declare fd_ed25519_verify,
   fd_ed25519_verify_batch_single_msg and fd_ed25519_strerror (fd_ed25519.h:96-101, :124-130, :137-138): any
   difference in a prototype, a result code or the fd_sha512_t tag is a compile error here.  The calls are
   what a verify tile makes (fd_verify_tile.h:92); nothing is linked or run. */
#include "ballet/ed25519/fd_ed25519.h"
#include "fd_ed25519_gpu.h"

int dropin_calls( uchar const * msg, ulong msg_sz, uchar const * sig, uchar const * pub, fd_sha512_t * sha,
                  fd_sha512_t * shas[ FD_ED25519_SIG_SZ ], uchar n );

int
dropin_calls( uchar const * msg, ulong msg_sz, uchar const * sig, uchar const * pub, fd_sha512_t * sha,
              fd_sha512_t * shas[ FD_ED25519_SIG_SZ ], uchar n ) {
  int (*one)( uchar const *, ulong, uchar const *, uchar const *, fd_sha512_t * ) = fd_ed25519_verify;
  int (*batch)( uchar const *, ulong const, uchar const *, uchar const *, fd_sha512_t **, uchar const ) =
      fd_ed25519_verify_batch_single_msg;
  int r = one( msg, msg_sz, sig, pub, sha );
  if( r == FD_ED25519_SUCCESS ) r = batch( msg, msg_sz, sig, pub, shas, n );
  return r == FD_ED25519_ERR_SIG || r == FD_ED25519_ERR_PUBKEY || r == FD_ED25519_ERR_MSG ? (int)fd_ed25519_strerror( r )[0] : r;
}
