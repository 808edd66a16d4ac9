/* ref_txn_harness.c -- TEST INFRASTRUCTURE ONLY.

   Driver compiled together with the reference's own transaction parser
   (src/ballet/txn/fd_txn_parse.c, taken in place from /root/reference by
   oracle/Makefile, never copied) into oracle/_ref/libfdref_txn.so: the
   checker that pins oracle/fd_txn_oracle.c and generates
   tests/golden/txn_parse.npz. */

#include "ballet/txn/fd_txn.h"

ulong
ref_txn_parse( uchar const * payload, ulong payload_sz, uchar * out ) {
  return fd_txn_parse( payload, payload_sz, out, NULL );
}

void
ref_txn_parse_batch( uchar const * arena, uint const * off, ushort const * sz, ulong n,
                     uchar * out, ulong stride, ushort * fp ) {
  for( ulong t=0UL; t<n; t++ ) fp[t] = (ushort)fd_txn_parse( arena + off[t], sz[t], out + t*stride, NULL );
}
