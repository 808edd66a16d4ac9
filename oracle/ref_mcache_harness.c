/* ref_mcache_harness.c -- TEST INFRASTRUCTURE ONLY.

   The reference's own mcache producer / consumer code, compiled in place
   from /root/reference by oracle/Makefile (never copied): the header-
   inline fd_mcache_publish (src/tango/mcache/fd_mcache.h:297-319), its
   AVX form fd_mcache_publish_avx (:351-367), fd_mcache_line_idx
   (:265-272), the FD_MCACHE_WAIT consumer macro (:451-545) and the
   fd_frag_meta_t layout and fd_frag_meta_ctl (src/tango/fd_tango_base.h:
   146-203, 280-300).  fd_mcache_new / fd_mcache_join live in fd_mcache.c,
   which logs through fd_log (the whole fd_util runtime); the one thing
   this harness restates is fd_mcache_new's line initialisation
   (src/tango/mcache/fd_mcache.c:60-66: line of seq0+i holds seq0+i-1,
   ctl = SOM|EOM|ERR), done with the reference's own inline helpers.
   libfdref_mcache.so lets tests/test_ref_mcache.py write a ring with the
   reference's publish and read it through fdgpu_mcache_wrap (the engine's
   handle on an existing fd_frag_meta_t ring), and drive the GPU verify
   tile from it (tests/test_gpu_vtile.py). */

#include "tango/mcache/fd_mcache.h"

ulong ref_frag_meta_sz( void ) { return sizeof(fd_frag_meta_t); }
ulong ref_mcache_align( void ) { return FD_MCACHE_ALIGN; }
ulong ref_mcache_line_idx( ulong seq, ulong depth ) { return fd_mcache_line_idx( seq, depth ); }

void
ref_mcache_init_lines( fd_frag_meta_t * mcache, ulong depth, ulong seq0 ) {
  ulong seq1 = fd_seq_inc( seq0, depth );
  for( ulong seq=seq0; seq!=seq1; seq=fd_seq_inc( seq, 1UL ) ) {
    fd_frag_meta_t * m = mcache + fd_mcache_line_idx( seq, depth );
    m->seq = fd_seq_dec( seq, 1UL );
    m->ctl = (ushort)fd_frag_meta_ctl( 0UL, 1, 1, 1 );
  }
}

void
ref_mcache_publish( fd_frag_meta_t * mcache, ulong depth, ulong seq, ulong sig, ulong chunk, ulong sz, ulong ctl,
                    ulong tsorig, ulong tspub, int avx ) {
#if FD_HAS_AVX
  if( avx ) { fd_mcache_publish_avx( mcache, depth, seq, sig, chunk, sz, ctl, tsorig, tspub ); return; }
#endif
  (void)avx;
  fd_mcache_publish( mcache, depth, seq, sig, chunk, sz, ctl, tsorig, tspub );
}

/* FD_MCACHE_WAIT with poll_max 2 (it counts the successful poll too; single-threaded, a seq not ready at
   the first poll is not ready at the second): 0 = frag seq read into *out, 1 = not yet published, -1 = overrun
   (*seq_found: the seq the line held) */
int
ref_mcache_wait( fd_frag_meta_t const * mcache, ulong depth, ulong seq, fd_frag_meta_t * out, ulong * seq_found ) {
  fd_frag_meta_t         meta[1];
  fd_frag_meta_t const * mline;
  ulong                  found;
  long                   diff;
  ulong                  poll_max = 2UL;
  FD_MCACHE_WAIT( meta, mline, found, diff, poll_max, mcache, depth, seq );
  (void)mline;
  if( !poll_max ) return 1;
  *seq_found = found;
  if( diff ) return -1;
  *out = meta[0];
  return 0;
}
