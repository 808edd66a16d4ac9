#pragma once
/* fd_gpu_sha512.h -- SHA-512 with one message per lane (CDNA4 device code).

   Replaces, for the verify path, the reference's k = SHA-512(R||A||M)
   computation: fd_sha512_init/append/fini (src/ballet/sha512/
   fd_sha512.c:265-398) over the AVX2 block core fd_sha512_core_avx2.S and
   the 4/8-lane AVX batch API (fd_sha512_batch_avx512.c).  Here every
   lane of a wave hashes its own signature's R||A||M: the 64-bit state
   words are VGPR pairs, rotations are v_alignbit_b32 pairs, Ch, Maj and
   the 3-way xors are v_bitop3_b32.  The message is read straight from the transaction payload
   (arbitrary byte alignment) with dword loads + v_alignbyte_b32; padding
   and the length block are synthesised in registers. */

#include "fd_gpu_f25519.h"

__constant__ u64 fd_gpu_sha512_k[ 80 ] = {
  0x428a2f98d728ae22UL, 0x7137449123ef65cdUL, 0xb5c0fbcfec4d3b2fUL, 0xe9b5dba58189dbbcUL,
  0x3956c25bf348b538UL, 0x59f111f1b605d019UL, 0x923f82a4af194f9bUL, 0xab1c5ed5da6d8118UL,
  0xd807aa98a3030242UL, 0x12835b0145706fbeUL, 0x243185be4ee4b28cUL, 0x550c7dc3d5ffb4e2UL,
  0x72be5d74f27b896fUL, 0x80deb1fe3b1696b1UL, 0x9bdc06a725c71235UL, 0xc19bf174cf692694UL,
  0xe49b69c19ef14ad2UL, 0xefbe4786384f25e3UL, 0x0fc19dc68b8cd5b5UL, 0x240ca1cc77ac9c65UL,
  0x2de92c6f592b0275UL, 0x4a7484aa6ea6e483UL, 0x5cb0a9dcbd41fbd4UL, 0x76f988da831153b5UL,
  0x983e5152ee66dfabUL, 0xa831c66d2db43210UL, 0xb00327c898fb213fUL, 0xbf597fc7beef0ee4UL,
  0xc6e00bf33da88fc2UL, 0xd5a79147930aa725UL, 0x06ca6351e003826fUL, 0x142929670a0e6e70UL,
  0x27b70a8546d22ffcUL, 0x2e1b21385c26c926UL, 0x4d2c6dfc5ac42aedUL, 0x53380d139d95b3dfUL,
  0x650a73548baf63deUL, 0x766a0abb3c77b2a8UL, 0x81c2c92e47edaee6UL, 0x92722c851482353bUL,
  0xa2bfe8a14cf10364UL, 0xa81a664bbc423001UL, 0xc24b8b70d0f89791UL, 0xc76c51a30654be30UL,
  0xd192e819d6ef5218UL, 0xd69906245565a910UL, 0xf40e35855771202aUL, 0x106aa07032bbd1b8UL,
  0x19a4c116b8d2d0c8UL, 0x1e376c085141ab53UL, 0x2748774cdf8eeb99UL, 0x34b0bcb5e19b48a8UL,
  0x391c0cb3c5c95a63UL, 0x4ed8aa4ae3418acbUL, 0x5b9cca4f7763e373UL, 0x682e6ff3d6b2b8a3UL,
  0x748f82ee5defb2fcUL, 0x78a5636f43172f60UL, 0x84c87814a1f0ab72UL, 0x8cc702081a6439ecUL,
  0x90befffa23631e28UL, 0xa4506cebde82bde9UL, 0xbef9a3f7b2c67915UL, 0xc67178f2e372532bUL,
  0xca273eceea26619cUL, 0xd186b8c721c0c207UL, 0xeada7dd6cde0eb1eUL, 0xf57d4f7fee6ed178UL,
  0x06f067aa72176fbaUL, 0x0a637dc5a2c898a6UL, 0x113f9804bef90daeUL, 0x1b710b35131c471bUL,
  0x28db77f523047d84UL, 0x32caab7b40c72493UL, 0x3c9ebe0a15c9bebcUL, 0x431d67c49c100d4cUL,
  0x4cc5d4becb3e42b6UL, 0x597f299cfc657e2aUL, 0x5fcb6fab3ad6faecUL, 0x6c44198c4a475817UL
};

/* 64-bit rotate / shift as two v_alignbit_b32 on the VGPR halves */
/* (hi:lo) as a bit cast of a 2-vector: written as (hi<<32)|lo the
   compiler splits later 64-bit adds into a low add and a high add */
typedef u32 fd_u32x2 __attribute__(( ext_vector_type( 2 ) ));
FD_DEV u64 fd_mk64( u32 lo, u32 hi ) { fd_u32x2 v = { lo, hi }; return __builtin_bit_cast( u64, v ); }
FD_DEV u64 fd_rotr64( u64 x, int n ) {
  u32 lo = (u32)x, hi = (u32)(x >> 32);
  if( n >= 32 ) { u32 t = lo; lo = hi; hi = t; n -= 32; }
  return fd_mk64( __builtin_amdgcn_alignbit( hi, lo, (u32)n ), __builtin_amdgcn_alignbit( lo, hi, (u32)n ) );
}
FD_DEV u64 fd_shr64( u64 x, int n ) {   /* n < 32 */
  u32 lo = (u32)x, hi = (u32)(x >> 32);
  return fd_mk64( __builtin_amdgcn_alignbit( hi, lo, (u32)n ), hi >> n );
}
FD_DEV u32 fd_bswap32( u32 x ) { return __builtin_bswap32( x ); }

/* Three-input boolean functions as one gfx950 v_bitop3_b32 per 32-bit
   half (truth table immediate: 0x96 = x^y^z, 0xe8 = majority).  The
   compiler leaves a 3-way xor as two v_xor_b32 per half. */
FD_DEV u64 fd_xor3_64( u64 x, u64 y, u64 z ) {
  return fd_mk64( __builtin_amdgcn_bitop3_b32( (u32)x, (u32)y, (u32)z, 0x96 ),
                  __builtin_amdgcn_bitop3_b32( (u32)(x>>32), (u32)(y>>32), (u32)(z>>32), 0x96 ) );
}
/* Ch(x, y, z) = x ? y : z as v_bitop3_b32 (truth table 0xca): the compiler's form is v_bfi_b32, which
   issues at half rate on gfx950 (4.25 cycles per wave64 instruction against 2.22 for v_bitop3_b32,
   profiles/r03/roofline/probe_r03b.txt) */
FD_DEV u64 fd_ch64( u64 x, u64 y, u64 z ) {
  return fd_mk64( __builtin_amdgcn_bitop3_b32( (u32)x, (u32)y, (u32)z, 0xca ),
                  __builtin_amdgcn_bitop3_b32( (u32)(x>>32), (u32)(y>>32), (u32)(z>>32), 0xca ) );
}
FD_DEV u64 fd_maj64( u64 x, u64 y, u64 z ) {
  return fd_mk64( __builtin_amdgcn_bitop3_b32( (u32)x, (u32)y, (u32)z, 0xe8 ),
                  __builtin_amdgcn_bitop3_b32( (u32)(x>>32), (u32)(y>>32), (u32)(z>>32), 0xe8 ) );
}

/* Load n32 consecutive little-endian 32-bit words starting at an
   arbitrary byte address p: aligned dword loads + v_alignbyte_b32.  Reads
   up to 4 bytes past p + 4*n32 (the batch arena carries tail slack). */
/* FD_SHA_LOAD (A/B knob): 1 plain loads, 0 loads with the non-temporal
   hint (the round-1 form).  Either way the compiler merges the
   dword-aligned word loads into global_load_dwordx4 (dword alignment
   suffices).  Measured on fd_hash_kernel, 1M x 1232-byte txns
   (profiles/r02/sha_ab): non-temporal 1.239 ms, FETCH_SIZE 1.60 GB (x2
   gfx950 correction: 3.27 GB = 2.5x the payload); plain 1.177 ms, 1.00 GB
   (2.05 GB = 1.6x): the hint let lines go before the lane's next quads. */
#ifndef FD_SHA_LOAD
#define FD_SHA_LOAD 1
#endif
template<int N32>
FD_DEV void fd_load_words( u32 w[ N32 ], unsigned char const * p ) {
  uintptr_t a  = (uintptr_t)p;
  u32 sh = (u32)( a & 3 );
  /* global address space: the caller's pointer is generic, and generic loads become flat_load
     (which wait on both the vector-memory and the LDS counters) */
  typedef __attribute__(( address_space( 1 ) )) u32 const gu32;
  gu32 * q = (gu32 *)( a & ~(uintptr_t)3 );
  u32 d[ N32 + 1 ];
#pragma unroll
  for( int i=0; i<N32+1; i++ ) {
#if FD_SHA_LOAD==0
    d[i] = __builtin_nontemporal_load( q + i );
#else
    d[i] = q[i];
#endif
  }
#pragma unroll
  for( int i=0; i<N32; i++ ) w[i] = __builtin_amdgcn_alignbyte( d[i+1], d[i], sh );
}

/* One 128-byte block.  A rolled loop over 5 groups of 16 unrolled rounds:
   the message schedule index is static inside a group (w[] stays in 32
   VGPRs) and the group's 16 round constants come from scalar loads, so
   neither the 80 constants nor the whole expanded schedule are ever live
   at once (a fully unrolled block needed ~200 VGPRs). */
#define FD_SHA512_ROUND( kt, wt ) do {                                              \
    u64 S1 = fd_xor3_64( fd_rotr64( e,14 ), fd_rotr64( e,18 ), fd_rotr64( e,41 ) ); \
    u64 ch = fd_ch64( e, f, g );                                                    \
    u64 t1 = hh + S1 + ch + (kt) + (wt);                                            \
    u64 S0 = fd_xor3_64( fd_rotr64( a,28 ), fd_rotr64( a,34 ), fd_rotr64( a,39 ) ); \
    u64 mj = fd_maj64( a, b, c );                                                   \
    hh = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + S0 + mj;      \
  } while(0)

FD_DEV void fd_sha512_block( u64 h[ 8 ], u64 w[ 16 ] ) {
  u64 a=h[0], b=h[1], c=h[2], d=h[3], e=h[4], f=h[5], g=h[6], hh=h[7];
#pragma unroll
  for( int r=0; r<16; r++ ) {
    FD_SHA512_ROUND( fd_gpu_sha512_k[r], w[r] );
    if( (r & 3)==3 ) __builtin_amdgcn_sched_barrier( 0 );
  }
#pragma unroll 1
  for( int grp=1; grp<5; grp++ ) {
    u64 const * kg = fd_gpu_sha512_k + 16*grp;
#pragma unroll
    for( int r=0; r<16; r++ ) {
      u64 w15 = w[(r+1)&15], w2 = w[(r+14)&15];
      u64 s0 = fd_xor3_64( fd_rotr64( w15, 1 ), fd_rotr64( w15, 8 ), fd_shr64( w15, 7 ) );
      u64 s1 = fd_xor3_64( fd_rotr64( w2, 19 ), fd_rotr64( w2, 61 ), fd_shr64( w2, 6 ) );
      w[r] += s0 + w[(r+9)&15] + s1;
      FD_SHA512_ROUND( kg[r], w[r] );
      if( (r & 3)==3 ) __builtin_amdgcn_sched_barrier( 0 );
    }
  }
  h[0]+=a; h[1]+=b; h[2]+=c; h[3]+=d; h[4]+=e; h[5]+=f; h[6]+=g; h[7]+=hh;
}

/* Message block b (of nb) of R || A || M with its padding and length, as 16 big-endian words; L = 64 + msg_sz
   input bytes.  R, A: the 32-byte encodings as 8 LE words; M: msg_sz bytes at msg. */
FD_DEV void fd_sha512_RAM_block( u64 w[ 16 ], u32 b, u32 nb, u32 L, u32 const R[ 8 ], u32 const A[ 8 ],
                                 unsigned char const * msg ) {
  u32 lw[32];
  if( b==0 ) {
#pragma unroll
    for( int i=0; i<8; i++ ) { lw[i] = R[i]; lw[8+i] = A[i]; }
    fd_load_words<16>( lw+16, msg );
  } else {
    fd_load_words<32>( lw, msg + (128u*b - 64u) );
  }
#pragma unroll
  for( int i=0; i<16; i++ ) w[i] = ((u64)fd_bswap32( lw[2*i] ) << 32) | (u64)fd_bswap32( lw[2*i+1] );
  if( 128u*(b+1u) > L ) {                       /* the message ends in this block: mask, pad, length */
#pragma unroll
    for( int i=0; i<16; i++ ) {
      /* mask bytes past the end, insert 0x80, insert the bit length */
      u64 x = w[i];
      int pos = (int)(128u*b) + 8*i;
      int nv  = (int)L - pos;                   /* valid bytes in this word */
      if( b==0 && i<8 ) nv = 8;                 /* R||A always present */
      u64 m = nv>=8 ? ~0UL : ( nv<=0 ? 0UL : ( ~0UL << (8*(8-nv)) ) );
      x &= m;
      if( nv>=0 && nv<8 ) x |= 0x80UL << (8*(7-nv));
      if( b==nb-1u && i==15 ) x = (u64)L << 3;
      if( b==nb-1u && i==14 ) x = 0UL;
      w[i] = x;
    }
  }
}

/* SHA-512( R || A || M ) -> 64-byte digest as 16 little-endian words
   (byte order of the digest, i.e. the scalar k's LE bytes).
   R, A: the 32-byte encodings as 8 LE words; M: msg_sz bytes at msg. */
FD_DEV void fd_sha512_RAM( u32 out[ 16 ], u32 const R[ 8 ], u32 const A[ 8 ],
                           unsigned char const * msg, u32 msg_sz ) {
  u64 h[8] = { 0x6a09e667f3bcc908UL, 0xbb67ae8584caa73bUL, 0x3c6ef372fe94f82bUL, 0xa54ff53a5f1d36f1UL,
               0x510e527fade682d1UL, 0x9b05688c2b3e6c1fUL, 0x1f83d9abfb41bd6bUL, 0x5be0cd19137e2179UL };
  u32 L  = 64u + msg_sz;              /* total input bytes */
  u32 nb = ( L + 17u + 127u ) >> 7;   /* blocks incl. padding + 128-bit length */
#pragma unroll 1
  for( u32 b=0; b<nb; b++ ) {
    u64 w[16];
    fd_sha512_RAM_block( w, b, nb, L, R, A, msg );
    fd_sha512_block( h, w );
  }
#pragma unroll
  for( int i=0; i<8; i++ ) { out[2*i] = fd_bswap32( (u32)(h[i] >> 32) ); out[2*i+1] = fd_bswap32( (u32)h[i] ); }
}

/* The same digest on a quad of lanes (the latency path's hash role: a batch that leaves SIMDs idle runs as
   long as its longest lane's instruction stream).  The rounds of a block depend on each other; its message
   schedule depends only on the block.  So the four lanes of a quad (q = 0..3, quad base lane qbase within
   the wave) each expand one block of a group of four into W_t + K_t (80 words, in registers), and then all
   four run the group's blocks' rounds in turn, block j's schedule read from lane qbase + j with
   ds_bpermute (issued four rounds ahead).  Per block the rounds' stream drops from 56 to 32 VALU
   instructions a round (rounds 16-79: no schedule and no K add); the expansions of four blocks cost the
   stream about what one block's schedule did.  All four lanes end with the digest. */
FD_DEV u64 fd_bperm64( u64 x, int addr ) {
  u32 lo = (u32)__builtin_amdgcn_ds_bpermute( addr, (int)(u32)x );
  u32 hi = (u32)__builtin_amdgcn_ds_bpermute( addr, (int)(u32)( x >> 32 ) );
  return fd_mk64( lo, hi );
}

#define FD_SHA512_ROUND_KW( kw ) do {                                               \
    u64 S1 = fd_xor3_64( fd_rotr64( e,14 ), fd_rotr64( e,18 ), fd_rotr64( e,41 ) ); \
    u64 ch = fd_ch64( e, f, g );                                                    \
    u64 t1 = hh + S1 + ch + (kw);                                                   \
    u64 S0 = fd_xor3_64( fd_rotr64( a,28 ), fd_rotr64( a,34 ), fd_rotr64( a,39 ) ); \
    u64 mj = fd_maj64( a, b, c );                                                   \
    hh = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + S0 + mj;      \
  } while(0)

FD_DEV void fd_sha512_RAM_quad( u32 out[ 16 ], u32 const R[ 8 ], u32 const A[ 8 ],
                                unsigned char const * msg, u32 msg_sz, u32 q, u32 qbase ) {
  u64 h[8] = { 0x6a09e667f3bcc908UL, 0xbb67ae8584caa73bUL, 0x3c6ef372fe94f82bUL, 0xa54ff53a5f1d36f1UL,
               0x510e527fade682d1UL, 0x9b05688c2b3e6c1fUL, 0x1f83d9abfb41bd6bUL, 0x5be0cd19137e2179UL };
  u32 L  = 64u + msg_sz;
  u32 nb = ( L + 17u + 127u ) >> 7;
#pragma unroll 1
  for( u32 g0=0; g0<nb; g0+=4u ) {
    u64 wk[80];
    {
      u32 bq = g0 + q;                          /* this lane's block of the group (none past the last) */
      u64 w[16];
      if( bq < nb ) fd_sha512_RAM_block( w, bq, nb, L, R, A, msg );
      else {
#pragma unroll
        for( int i=0; i<16; i++ ) w[i] = 0UL;
      }
#pragma unroll
      for( int t=0; t<16; t++ ) wk[t] = w[t];
#pragma unroll
      for( int t=16; t<80; t++ ) {
        u64 w15 = wk[t-15], w2 = wk[t-2];
        u64 s0 = fd_xor3_64( fd_rotr64( w15, 1 ), fd_rotr64( w15, 8 ), fd_shr64( w15, 7 ) );
        u64 s1 = fd_xor3_64( fd_rotr64( w2, 19 ), fd_rotr64( w2, 61 ), fd_shr64( w2, 6 ) );
        wk[t] = wk[t-16] + s0 + wk[t-7] + s1;
      }
#pragma unroll
      for( int t=0; t<80; t++ ) wk[t] += fd_gpu_sha512_k[t];
    }
#pragma unroll 1
    for( u32 j=0; j<4u && g0+j<nb; j++ ) {      /* (nb is the quad's: its four lanes agree) */
      int addr = (int)( ( qbase + j ) << 2 );
      u64 a=h[0], b=h[1], c=h[2], d=h[3], e=h[4], f=h[5], g=h[6], hh=h[7];
      u64 pf[4];
#pragma unroll
      for( int t=0; t<4; t++ ) pf[t] = fd_bperm64( wk[t], addr );
#pragma unroll
      for( int t=0; t<80; t++ ) {
        u64 kw = pf[t & 3];
        if( t + 4 < 80 ) pf[t & 3] = fd_bperm64( wk[t + 4], addr );
        FD_SHA512_ROUND_KW( kw );
        if( (t & 3)==3 ) __builtin_amdgcn_sched_barrier( 0 );
      }
      h[0]+=a; h[1]+=b; h[2]+=c; h[3]+=d; h[4]+=e; h[5]+=f; h[6]+=g; h[7]+=hh;
    }
  }
#pragma unroll
  for( int i=0; i<8; i++ ) { out[2*i] = fd_bswap32( (u32)(h[i] >> 32) ); out[2*i+1] = fd_bswap32( (u32)h[i] ); }
}

/* SHA-512( M ) of msg_sz bytes at msg (any alignment) -> digest bytes as
   16 words in digest byte order.  Reads up to 132 bytes past the last
   whole block of the message; the caller's buffer carries that slack. */
FD_DEV void fd_sha512_bytes( u32 out[ 16 ], unsigned char const * msg, u32 msg_sz ) {
  u64 h[8] = { 0x6a09e667f3bcc908UL, 0xbb67ae8584caa73bUL, 0x3c6ef372fe94f82bUL, 0xa54ff53a5f1d36f1UL,
               0x510e527fade682d1UL, 0x9b05688c2b3e6c1fUL, 0x1f83d9abfb41bd6bUL, 0x5be0cd19137e2179UL };
  u32 L  = msg_sz;
  u32 nb = ( L + 17u + 127u ) >> 7;
#pragma unroll 1
  for( u32 b=0; b<nb; b++ ) {
    u64 w[16];
    u32 lw[32];
    /* blocks wholly past the message (the last one or two: padding and
       length only) read nothing */
    if( 128u*b < L ) fd_load_words<32>( lw, msg + 128u*b );
    else {
#pragma unroll
      for( int i=0; i<32; i++ ) lw[i] = 0u;
    }
#pragma unroll
    for( int i=0; i<16; i++ ) {
      u64 x = ((u64)fd_bswap32( lw[2*i] ) << 32) | (u64)fd_bswap32( lw[2*i+1] );
      int pos = (int)(128u*b) + 8*i;
      int nv  = (int)L - pos;
      u64 m = nv>=8 ? ~0UL : ( nv<=0 ? 0UL : ( ~0UL << (8*(8-nv)) ) );
      x &= m;
      if( nv>=0 && nv<8 ) x |= 0x80UL << (8*(7-nv));
      if( b==nb-1u && i==15 ) x = (u64)L << 3;
      if( b==nb-1u && i==14 ) x = 0UL;
      w[i] = x;
    }
    fd_sha512_block( h, w );
  }
#pragma unroll
  for( int i=0; i<8; i++ ) { out[2*i] = fd_bswap32( (u32)(h[i] >> 32) ); out[2*i+1] = fd_bswap32( (u32)h[i] ); }
}

