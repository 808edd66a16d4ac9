/* dump_vectors.c -- TEST INFRASTRUCTURE ONLY.

   Compiled by oracle/Makefile against the reference's known-answer
   vector tables (read in place from /root/reference; never copied) and
   run once in the build container to export them as data for
   tests/golden/gen_golden.py.  Output: one line per vector,
     <set> <tc_id> <ok> <msg_hex|-> <pub_hex> <sig_hex>
   Sets: cctv (src/ballet/ed25519/test_ed25519_cctv.c, 914 vectors),
   wycheproof (src/ballet/ed25519/test_ed25519_wycheproof.c, 133). */

#include <stdio.h>
#include "ballet/ed25519/test_ed25519_cctv.c"
#include "ballet/ed25519/test_ed25519_wycheproof.c"

static void
hex( uchar const * p, ulong n ) {
  if( !n ) { putchar( '-' ); return; }
  for( ulong i=0; i<n; i++ ) printf( "%02x", p[i] );
}

#define DUMP( set, arr ) do {                                               \
    for( ulong i=0UL; i<sizeof(arr)/sizeof(arr[0]) && arr[i].comment; i++ ) {  \
      printf( "%s %u %d ", set, arr[i].tc_id, arr[i].ok );                   \
      hex( arr[i].msg, arr[i].msg_sz ); putchar( ' ' );                      \
      hex( arr[i].pub, 32 ); putchar( ' ' );                                 \
      hex( arr[i].sig, 64 ); putchar( '\n' );                                \
    }                                                                        \
  } while(0)

int
main( void ) {
  DUMP( "cctv",       ed25519_verify_cctvs );
  DUMP( "wycheproof", ed25519_verify_wycheproofs );
  return 0;
}
