/* vtile_sandbox: the GPU verify tile under a seccomp filter.

   The reference runs every tile under seccomp after privileged_init
   (src/disco/topo/fd_topo_run.c:98-136; the verify tile allows only
   write / fsync, src/disco/verify/fd_verify_tile.seccomppolicy).  A GPU
   verify tile keeps talking to the kernel driver after init, so its
   policy is longer.  This program finds and checks that policy:

     privileged init   open the GPU (HIP runtime init), create the tile
                       (fdgpu_vtile_new_opts: engine contexts, pinned
                       out dcache, tcache), an in mcache + a registered
                       in dcache holding signed fd_txn_m_t records, and
                       run one batch through the zero-copy intake
                       unfiltered (lazy runtime init: code objects,
                       queues, the gather stream);
     sandbox           no_new_privs + a seccomp BPF filter on every
                       thread of the process (SECCOMP_FILTER_FLAG_TSYNC:
                       the HIP runtime's own threads too);
     run               a second batch (fresh seqs and transactions) under
                       the filter; every frag must come back PUBLISH.

   discover  the filter allows a base set and traps everything else; the
             SIGSYS handler counts the syscall and re-issues it from a
             trampoline whose address the filter allows, so the run goes
             on and every syscall the tile makes after init is listed;
   enforce   the filter allows exactly the policy (syscall numbers, and
             ioctl only on the driver's descriptors: /dev/kfd and the
             DRM render node, found before the filter goes on); anything
             else traps, and the handler names the syscall and exits 3.

   usage: vtile_sandbox discover|enforce [--launcher] [syscall ...]
          (enforce: the allowed syscall names, e.g. from the policy file)
   The tile runs with the bench's paced-tile defaults: two engine contexts,
   latency-path workgroups alone on their CUs (cu_exclusive) within each
   context's CU share (lat_share), 16 CUs reserved for the copies;
   --launcher adds its launch thread (fdgpu_vtile_opts_t.launcher).  The
   filter covers every thread (TSYNC): the HIP runtime's, the launch thread.

   Served form (include/fd_verify_gpu.h, fdgpu_vsvc_*): the verify tile is a
   process with no GPU context, its GPU's verify service another process.
     vtile_sandbox served discover|enforce [--launcher] [tile syscall ...] -- [service syscall ...]
   forks the tile process before the service touches the GPU (the two share
   the in link and the service segment), runs the warm-up batch unfiltered,
   then puts the tile under its filter (discover, or enforce of the names
   before "--") and the service under its own (discover when no names follow
   "--", else enforce of them) and runs the second batch.  Prints one JSON
   line per process (role "tile" / "service").

   Prints one JSON line.  Needs libfdgpu_vtile.so, libfdgpu_ed25519.so
   and libfdsynth.so (LD_LIBRARY_PATH=firedancer_amd). */

#define _GNU_SOURCE
#include <dirent.h>
#include <errno.h>
#include <linux/audit.h>
#include <linux/filter.h>
#include <linux/seccomp.h>
#include <signal.h>
#include <stddef.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <stdatomic.h>
#include <sys/mman.h>
#include <sys/prctl.h>
#include <sys/syscall.h>
#include <time.h>
#include <ucontext.h>
#include <unistd.h>

#include "../../include/fd_verify_gpu.h"

typedef unsigned char uchar;
typedef unsigned long ulong;

/* libfdsynth.so (firedancer_amd/csrc/fd_synth.c) */
typedef struct { uint8_t prv[32], pub[32], s[32], prefix[32]; } fdsynth_key_t;
void   fdsynth_keys( fdsynth_key_t * keys, size_t n, uint64_t seed );
size_t fdsynth_txns( uint8_t * payload, size_t stride, fdgpu_txn_desc_t * desc, int8_t * expect, size_t n,
                     int kind, int max_signers, double invalid_frac, uint64_t seed,
                     fdsynth_key_t const * keys, size_t nkeys, int threads );

#define N_FRAG   4096UL          /* frags per batch */
#define REC_SZ   1408UL          /* one fd_txn_m_t record (80 + 1232 B) rounded to chunk pairs */
#define MAX_NR   512

/* ---- syscall names (from the kernel headers, read before the filter goes on) ---- */

static char g_name[ MAX_NR ][ 32 ];

static void
load_names( void ) {
  FILE * f = fopen( "/usr/include/x86_64-linux-gnu/asm/unistd_64.h", "r" );
  if( !f ) f = fopen( "/usr/include/asm/unistd_64.h", "r" );
  if( !f ) return;
  char line[ 256 ], nm[ 64 ]; int nr;
  while( fgets( line, sizeof(line), f ) )
    if( sscanf( line, "#define __NR_%63s %d", nm, &nr ) == 2 && nr >= 0 && nr < MAX_NR )
      snprintf( g_name[ nr ], sizeof(g_name[ nr ]), "%s", nm );
  fclose( f );
}

static int
nr_of( char const * name ) {
  for( int i=0; i<MAX_NR; i++ ) if( !strcmp( g_name[i], name ) ) return i;
  return -1;
}

/* ---- the trampoline: syscalls issued from here pass the discovery filter ---- */

long fdsb_tramp( long nr, long a0, long a1, long a2, long a3, long a4, long a5 );
extern char fdsb_tramp_begin[], fdsb_tramp_end[];
__asm__(
  ".text\n"
  ".balign 64\n"
  ".globl fdsb_tramp_begin\n"
  "fdsb_tramp_begin:\n"
  ".globl fdsb_tramp\n"
  ".type fdsb_tramp, @function\n"
  "fdsb_tramp:\n"
  "  mov %rdi, %rax\n"
  "  mov %rsi, %rdi\n"
  "  mov %rdx, %rsi\n"
  "  mov %rcx, %rdx\n"
  "  mov %r8, %r10\n"
  "  mov %r9, %r8\n"
  "  mov 8(%rsp), %r9\n"
  "  syscall\n"
  "  ret\n"
  ".globl fdsb_tramp_end\n"
  "fdsb_tramp_end:\n" );

static volatile unsigned long g_count[ MAX_NR ];
static int g_enforce;

static void
put( char const * s ) { fdsb_tramp( SYS_write, 2, (long)s, (long)strlen( s ), 0, 0, 0 ); }

static void
on_sigsys( int sig, siginfo_t * si, void * uc_ ) {
  (void)sig;
  ucontext_t * uc = (ucontext_t *)uc_;
  int nr = si->si_syscall;
  if( g_enforce ) {                       /* name the blocked syscall and stop */
    char msg[ 128 ];
    char const * nm = ( nr >= 0 && nr < MAX_NR && g_name[nr][0] ) ? g_name[nr] : "?";
    int n = 0;
    msg[n++] = '{';
    char const * a = "\"blocked_syscall\": \"";
    while( *a ) msg[n++] = *a++;
    while( *nm && n < 100 ) msg[n++] = *nm++;
    msg[n++] = '"'; msg[n++] = '}'; msg[n++] = '\n'; msg[n] = 0;
    put( msg );
    fdsb_tramp( SYS_exit_group, 3, 0, 0, 0, 0, 0 );
  }
  if( nr >= 0 && nr < MAX_NR ) __atomic_fetch_add( &g_count[ nr ], 1UL, __ATOMIC_RELAXED );
  greg_t * g = uc->uc_mcontext.gregs;
  g[ REG_RAX ] = fdsb_tramp( nr, g[ REG_RDI ], g[ REG_RSI ], g[ REG_RDX ], g[ REG_R10 ], g[ REG_R8 ], g[ REG_R9 ] );
}

/* ---- BPF ---- */

#define MAX_INS 256
static struct sock_filter g_prog[ MAX_INS ];
static int g_nins;
static void emit( struct sock_filter f ) { if( g_nins < MAX_INS ) g_prog[ g_nins++ ] = f; }

#define LD_NR    BPF_STMT( BPF_LD | BPF_W | BPF_ABS, offsetof( struct seccomp_data, nr ) )
#define RET(x)   BPF_STMT( BPF_RET | BPF_K, (x) )

/* allow[]: syscall numbers allowed outright; ioctl (if in allow_ioctl) only on fds[] */
static int
install( int const * allow, int n_allow, int ioctl_ok, int const * fds, int n_fds ) {
  g_nins = 0;
  emit( (struct sock_filter)BPF_STMT( BPF_LD | BPF_W | BPF_ABS, offsetof( struct seccomp_data, arch ) ) );
  emit( (struct sock_filter)BPF_JUMP( BPF_JMP | BPF_JEQ | BPF_K, AUDIT_ARCH_X86_64, 1, 0 ) );
  emit( (struct sock_filter)RET( SECCOMP_RET_KILL_PROCESS ) );
  {                                       /* the trampoline's own syscalls (only the SIGSYS handler uses it) */
    uintptr_t lo = (uintptr_t)fdsb_tramp_begin, hi = (uintptr_t)fdsb_tramp_end;
    if( ( lo >> 32 ) != ( hi >> 32 ) ) return -1;
    emit( (struct sock_filter)BPF_STMT( BPF_LD | BPF_W | BPF_ABS, offsetof( struct seccomp_data, instruction_pointer ) + 4 ) );
    emit( (struct sock_filter)BPF_JUMP( BPF_JMP | BPF_JEQ | BPF_K, (uint32_t)( lo >> 32 ), 0, 4 ) );
    emit( (struct sock_filter)BPF_STMT( BPF_LD | BPF_W | BPF_ABS, offsetof( struct seccomp_data, instruction_pointer ) ) );
    emit( (struct sock_filter)BPF_JUMP( BPF_JMP | BPF_JGE | BPF_K, (uint32_t)lo, 0, 2 ) );
    emit( (struct sock_filter)BPF_JUMP( BPF_JMP | BPF_JGT | BPF_K, (uint32_t)hi, 1, 0 ) );
    emit( (struct sock_filter)RET( SECCOMP_RET_ALLOW ) );
  }
  emit( (struct sock_filter)LD_NR );
  for( int i=0; i<n_allow; i++ ) {
    emit( (struct sock_filter)BPF_JUMP( BPF_JMP | BPF_JEQ | BPF_K, (uint32_t)allow[i], 0, 1 ) );
    emit( (struct sock_filter)RET( SECCOMP_RET_ALLOW ) );
  }
  if( ioctl_ok ) {                        /* ioctl( fd, ... ) with fd one of the driver's */
    emit( (struct sock_filter)BPF_JUMP( BPF_JMP | BPF_JEQ | BPF_K, SYS_ioctl, 0, (uint8_t)( 2 + 2*n_fds ) ) );
    emit( (struct sock_filter)BPF_STMT( BPF_LD | BPF_W | BPF_ABS, offsetof( struct seccomp_data, args[0] ) ) );
    for( int i=0; i<n_fds; i++ ) {
      emit( (struct sock_filter)BPF_JUMP( BPF_JMP | BPF_JEQ | BPF_K, (uint32_t)fds[i], 0, 1 ) );
      emit( (struct sock_filter)RET( SECCOMP_RET_ALLOW ) );
    }
    emit( (struct sock_filter)RET( SECCOMP_RET_TRAP ) );
  }
  emit( (struct sock_filter)RET( SECCOMP_RET_TRAP ) );
  if( g_nins >= MAX_INS ) return -1;
  struct sock_fprog prog = { .len = (unsigned short)g_nins, .filter = g_prog };
  if( prctl( PR_SET_NO_NEW_PRIVS, 1, 0, 0, 0 ) ) return -2;
  long r = syscall( SYS_seccomp, SECCOMP_SET_MODE_FILTER, SECCOMP_FILTER_FLAG_TSYNC, &prog );
  return r == 0 ? 0 : (int)( r > 0 ? -4 : -3 );   /* > 0: the id of a thread that could not be synced */
}

/* the driver's descriptors: /dev/kfd and the DRM nodes under /dev/dri */
static int
driver_fds( int * fds, int max ) {
  int n = 0;
  DIR * d = opendir( "/proc/self/fd" );
  if( !d ) return 0;
  struct dirent * e;
  while( ( e = readdir( d ) ) && n < max ) {
    char p[ 320 ], t[ 256 ];
    snprintf( p, sizeof(p), "/proc/self/fd/%s", e->d_name );
    ssize_t k = readlink( p, t, sizeof(t) - 1 );
    if( k <= 0 ) continue;
    t[k] = 0;
    if( !strcmp( t, "/dev/kfd" ) || !strncmp( t, "/dev/dri/", 9 ) ) fds[ n++ ] = atoi( e->d_name );
  }
  closedir( d );
  return n;
}

/* ---- one batch through the tile ---- */

static ulong
now_ns( void ) { struct timespec ts; clock_gettime( CLOCK_MONOTONIC, &ts ); return (ulong)ts.tv_sec*1000000000UL + (ulong)ts.tv_nsec; }

static int
run_batch( fdgpu_vtile_t * vt, fdgpu_mcache_t * mc, uchar * dcache, uchar const * payload, fdgpu_txn_desc_t const * desc,
           ulong seq0, ulong * published ) {
  for( ulong i=0; i<N_FRAG; i++ ) {
    ulong chunk = ( ( seq0 + i ) % ( 2UL*N_FRAG ) ) * ( REC_SZ / FDGPU_CHUNK_SZ );
    uchar * rec = dcache + chunk * FDGPU_CHUNK_SZ;
    memset( rec, 0, FDGPU_TXNM_HDR_SZ );
    ((fdgpu_txnm_t *)rec)->payload_sz = desc[i].payload_sz;
    memcpy( rec + FDGPU_TXNM_HDR_SZ, payload + desc[i].payload_off, desc[i].payload_sz );
    ulong sz = FDGPU_TXNM_HDR_SZ + desc[i].payload_sz;
    ulong ts = now_ns();
    fdgpu_mcache_publish( mc, seq0 + i, 0UL, (unsigned)chunk, (unsigned)sz, ts, ts );
    int rc;
    while( ( rc = fdgpu_vtile_during_frag( vt, 0UL, rec, sz, seq0 + i, ts ) ) == -2 ) {
      fdgpu_vtile_done_t d[ 64 ];
      ulong k = fdgpu_vtile_after_frags( vt, d, 64, 1 );
      for( ulong j=0; j<k; j++ ) *published += d[j].result == FDGPU_VTILE_PUBLISH;
    }
    if( rc ) return rc;
    if( ( i & 511UL ) == 511UL ) fdgpu_vtile_housekeep( vt, 1 );   /* early GPU copies and partial launches too */
  }
  if( fdgpu_vtile_flush( vt ) ) return -10;
  static fdgpu_vtile_done_t d[ N_FRAG ];
  ulong t0 = now_ns();
  while( fdgpu_vtile_pending( vt ) ) {
    ulong k = fdgpu_vtile_after_frags( vt, d, N_FRAG, 1 );
    for( ulong j=0; j<k; j++ ) *published += d[j].result == FDGPU_VTILE_PUBLISH;
    if( now_ns() - t0 > 20000000000UL ) return -11;
  }
  return 0;
}

/* the JSON report of a run under the filter (stdout writes are syscalls too: counted after the snapshot) */
static void
report( char const * role, char const * mode, int rc, ulong frags, ulong published, ulong dt, int n_fds, char const * extra ) {
  unsigned long snap[ MAX_NR ];
  for( int i=0; i<MAX_NR; i++ ) snap[i] = g_count[i];
  char buf[ 8192 ]; int n = 0;
  n += snprintf( buf + n, sizeof(buf) - n, "{\"role\": \"%s\", \"mode\": \"%s\", \"rc\": %d, \"frags\": %lu, \"published\": %lu, "
                 "\"batch_ms\": %.3f, \"driver_fds\": %d, \"filter_instructions\": %d, %s\"syscalls_after_init\": {",
                 role, mode, rc, frags, published, (double)dt * 1e-6, n_fds, g_nins, extra );
  int first = 1;
  for( int i=0; i<MAX_NR; i++ ) if( snap[i] ) {
    n += snprintf( buf + n, sizeof(buf) - n, "%s\"%s\": %lu", first ? "" : ", ", g_name[i][0] ? g_name[i] : "?", snap[i] );
    first = 0;
  }
  n += snprintf( buf + n, sizeof(buf) - n, "}}\n" );
  fdsb_tramp( SYS_write, 1, (long)buf, (long)n, 0, 0, 0 );   /* (the harness's own output: not counted, not filtered) */
}

static int
names_to_nrs( char ** names, int n, int * allow, int * ioctl_ok ) {
  int k = 0;
  for( int i=0; i<n; i++ ) {
    if( !strcmp( names[i], "ioctl" ) ) { *ioctl_ok = 1; continue; }
    int nr = nr_of( names[i] );
    if( nr < 0 ) { printf( "{\"error\": \"unknown syscall %s\"}\n", names[i] ); return -1; }
    allow[ k++ ] = nr;
  }
  return k;
}

static int
base_set( int * allow ) {               /* discover: what the handler itself and the process teardown need */
  char const * base[] = { "rt_sigreturn", "exit", "exit_group" };
  int k = 0;
  for( unsigned i=0; i<sizeof(base)/sizeof(base[0]); i++ ) { int nr = nr_of( base[i] ); if( nr >= 0 ) allow[ k++ ] = nr; }
  return k;
}

/* ---- the served form: a tile process without a GPU context, its verify service ---- */

typedef struct { _Atomic int phase; _Atomic int tile_rc; } served_ctl_t;   /* phase: 1 warm-up done, 2 tile done */

static int
served_main( int argc, char ** argv, int launcher ) {
  int i = 2;
  int tile_discover = !strcmp( argv[i++], "discover" );
  while( i < argc && !strncmp( argv[i], "--", 2 ) && argv[i][2] ) i++;       /* (options, parsed by main) */
  char ** tnames = argv + i; int ntn = 0;
  while( i < argc && strcmp( argv[i], "--" ) ) { i++; ntn++; }
  char ** snames = NULL; int nsn = 0;
  if( i < argc ) { snames = argv + i + 1; nsn = argc - i - 1; }
  int svc_discover = nsn == 0;

  /* privileged init, before anything touches the GPU: the payloads, the in link (mcache lines + in dcache in
     shared memory: the tile process is the producer and the tile, the service's GPU reads the records) */
  static fdsynth_key_t keys[ 64 ];
  fdsynth_keys( keys, 64, 77 );
  uchar * payload = (uchar *)malloc( 2*N_FRAG*1232UL + 1024UL );
  fdgpu_txn_desc_t * desc = (fdgpu_txn_desc_t *)calloc( 2*N_FRAG, sizeof(fdgpu_txn_desc_t) );
  int8_t * expect = (int8_t *)calloc( 2*N_FRAG, 1 );
  fdsynth_txns( payload, 1232UL, desc, expect, 2*N_FRAG, 0, 1, 0.0, 4242UL, keys, 64, 4 );
  ulong depth = 4UL*N_FRAG, dsz = 2UL*N_FRAG*REC_SZ, lsz = ( depth * 32UL + 4095UL ) & ~4095UL;
  uchar * dc = (uchar *)mmap( NULL, dsz, PROT_READ | PROT_WRITE, MAP_SHARED | MAP_ANONYMOUS, -1, 0 );
  void * lines = mmap( NULL, lsz, PROT_READ | PROT_WRITE, MAP_SHARED | MAP_ANONYMOUS, -1, 0 );
  served_ctl_t * ctl = (served_ctl_t *)mmap( NULL, 4096, PROT_READ | PROT_WRITE, MAP_SHARED | MAP_ANONYMOUS, -1, 0 );
  if( dc == MAP_FAILED || lines == MAP_FAILED || ctl == MAP_FAILED ) { printf( "{\"error\": \"mmap\"}\n" ); return 1; }
  fdgpu_mcache_t * tmp = fdgpu_mcache_new( depth, 0UL );           /* lines initialised "one lap behind" */
  memcpy( lines, fdgpu_mcache_lines( tmp ), depth * 32UL );
  fdgpu_mcache_delete( tmp );
  fdgpu_vsvc_cfg_t cfg; memset( &cfg, 0, sizeof(cfg) );
  cfg.clients = 1; cfg.out_dcache_bytes = 8UL*N_FRAG*REC_SZ; cfg.batch_txn = N_FRAG; cfg.max_inflight = 1; cfg.nctx = 2;
  cfg.gather_cus = 16; cfg.launcher = launcher;
  fdgpu_vsvc_t * svc = fdgpu_vsvc_new( NULL, &cfg );
  if( !svc || fdgpu_vsvc_add_region( svc, 0, dc, dsz ) || fdgpu_vsvc_add_region( svc, 1, lines, lsz ) ) {
    printf( "{\"error\": \"service segment\"}\n" ); return 1;
  }
  fflush( stdout ); fflush( stderr );
  pid_t pid = fork();
  if( pid < 0 ) { printf( "{\"error\": \"fork\"}\n" ); return 1; }
  if( pid == 0 ) {                                        /* ---- the tile process: no GPU call ---- */
    fdgpu_mcache_t * mc = fdgpu_mcache_wrap( lines, depth );
    fdgpu_vtile_opts_t opt; memset( &opt, 0, sizeof(opt) );
    fdgpu_vtile_t * vt = fdgpu_vtile_new_svc( svc, 0, 1UL << 16, 99UL, &opt );
    if( !mc || !vt || fdgpu_vtile_set_svc_region( vt, 0, dc, dsz ) || fdgpu_vtile_set_svc_region( vt, 1, lines, lsz ) ||
        fdgpu_vtile_set_in_link( vt, mc ) ) { printf( "{\"role\": \"tile\", \"error\": \"init\"}\n" ); _exit( 1 ); }
    ulong pub0 = 0UL, pub1 = 0UL;
    int rc = run_batch( vt, mc, dc, payload, desc, 0UL, &pub0 );       /* (waits for the service's verdicts) */
    if( rc || pub0 != N_FRAG ) { printf( "{\"role\": \"tile\", \"error\": \"warm-up rc %d published %lu\"}\n", rc, pub0 ); _exit( 1 ); }
    int fds[ 16 ]; int n_fds = driver_fds( fds, 16 );                  /* (none: no GPU context here) */
    int allow[ MAX_NR ], n_allow = 0, ioctl_ok = 0;
    n_allow = tile_discover ? base_set( allow ) : names_to_nrs( tnames, ntn, allow, &ioctl_ok );
    if( n_allow < 0 ) _exit( 1 );
    struct sigaction sa; memset( &sa, 0, sizeof(sa) );
    sa.sa_sigaction = on_sigsys; sa.sa_flags = SA_SIGINFO;
    sigaction( SIGSYS, &sa, NULL );
    g_enforce = !tile_discover;
    fflush( stdout );
    atomic_store( &ctl->phase, 1 );                                      /* the service may go under its filter */
    while( atomic_load( &ctl->phase ) < 2 ) ;                             /* ... and has */
    if( ( rc = install( allow, n_allow, ioctl_ok, fds, n_fds ) ) ) { printf( "{\"role\": \"tile\", \"error\": \"seccomp %d\"}\n", rc ); _exit( 1 ); }
    ulong t0 = now_ns();
    rc = run_batch( vt, mc, dc, payload, desc + N_FRAG, N_FRAG, &pub1 );
    ulong dt = now_ns() - t0;
    report( "tile", tile_discover ? "discover" : "enforce", rc, N_FRAG, pub1, dt, n_fds, "\"gpu_open\": 0, " );
    atomic_store( &ctl->tile_rc, rc || pub1 != N_FRAG ? 1 : 0 );
    atomic_store( &ctl->phase, 3 );
    fdsb_tramp( SYS_exit_group, 0, 0, 0, 0, 0, 0 );           /* (the harness's exit: the tile itself never exits) */
  }
  /* ---- the verify service: the GPU ---- */
  if( fdgpu_vsvc_start( svc, 0 ) ) { printf( "{\"role\": \"service\", \"error\": \"start: %s\"}\n", fdgpu_last_error() ); return 1; }
  while( atomic_load( &ctl->phase ) < 1 ) fdgpu_vsvc_poll( svc );        /* the warm-up batch */
  int fds[ 16 ]; int n_fds = driver_fds( fds, 16 );
  int allow[ MAX_NR ], n_allow = 0, ioctl_ok = 0;
  n_allow = svc_discover ? base_set( allow ) : names_to_nrs( snames, nsn, allow, &ioctl_ok );
  if( n_allow < 0 ) return 1;
  struct sigaction sa; memset( &sa, 0, sizeof(sa) );
  sa.sa_sigaction = on_sigsys; sa.sa_flags = SA_SIGINFO;
  sigaction( SIGSYS, &sa, NULL );
  g_enforce = !svc_discover;
  fflush( stdout ); fflush( stderr );
  int rc = install( allow, n_allow, ioctl_ok, fds, n_fds );
  if( rc ) { printf( "{\"role\": \"service\", \"error\": \"seccomp %d\"}\n", rc ); return 1; }
  atomic_store( &ctl->phase, 2 );
  ulong t0 = now_ns();
  while( atomic_load( &ctl->phase ) < 3 && now_ns() - t0 < 30000000000UL ) fdgpu_vsvc_poll( svc );
  ulong dt = now_ns() - t0;
  fdgpu_vsvc_stats_t st; fdgpu_vsvc_stats( svc, &st );
  char extra[ 160 ];
  snprintf( extra, sizeof(extra), "\"launcher\": %d, \"completed\": %lu, \"batches\": %lu, ", launcher, st.completed, st.gm.batches );
  report( "service", svc_discover ? "discover" : "enforce", atomic_load( &ctl->phase ) < 3 ? -12 : atomic_load( &ctl->tile_rc ),
          st.completed, st.completed, dt, n_fds, extra );
  fdsb_tramp( SYS_exit_group, atomic_load( &ctl->phase ) < 3 || atomic_load( &ctl->tile_rc ) ? 1 : 0, 0, 0, 0, 0, 0 );
  return 0;
}

int
main( int argc, char ** argv ) {
  int launcher = 0;
  for( int i=1; i<argc; i++ ) if( !strcmp( argv[i], "--launcher" ) ) launcher = 1;
  load_names();
  if( argc >= 3 && !strcmp( argv[1], "served" ) && ( !strcmp( argv[2], "discover" ) || !strcmp( argv[2], "enforce" ) ) )
    return served_main( argc, argv, launcher );
  if( argc < 2 || ( strcmp( argv[1], "discover" ) && strcmp( argv[1], "enforce" ) ) ) {
    fprintf( stderr, "usage: %s discover|enforce [--launcher] [syscall ...]\n"
                     "       %s served discover|enforce [--launcher] [tile syscall ...] -- [service syscall ...]\n", argv[0], argv[0] );
    return 2;
  }
  int discover = !strcmp( argv[1], "discover" );

  /* ---- privileged init ---- */
  static fdsynth_key_t keys[ 64 ];
  fdsynth_keys( keys, 64, 77 );
  uchar * payload = (uchar *)malloc( 2*N_FRAG*1232UL + 1024UL );
  fdgpu_txn_desc_t * desc = (fdgpu_txn_desc_t *)calloc( 2*N_FRAG, sizeof(fdgpu_txn_desc_t) );
  int8_t * expect = (int8_t *)calloc( 2*N_FRAG, 1 );
  fdsynth_txns( payload, 1232UL, desc, expect, 2*N_FRAG, 0 /* LARGE_NOOP */, 1, 0.0, 4242UL, keys, 64, 4 );
  fdgpu_mcache_t * mc = fdgpu_mcache_new( 4UL*N_FRAG, 0UL );
  uchar * dcache = (uchar *)fdgpu_host_alloc( 2UL*N_FRAG*REC_SZ );
  /* the bench's paced tile: two contexts, exclusive latency-path workgroups within each context's CU share (the
     defaults), 16 CUs for the copies, and (--launcher) its launch thread */
  fdgpu_vtile_opts_t opt; memset( &opt, 0, sizeof(opt) ); opt.nctx = 2; opt.gather_cus = 16; opt.launcher = launcher;
  fdgpu_vtile_t * vt = fdgpu_vtile_new_opts( 0, N_FRAG, 1UL << 16, 99UL, 8UL*N_FRAG*REC_SZ, 0, &opt );
  if( !mc || !dcache || !vt || fdgpu_vtile_set_in_link( vt, mc ) ) {
    printf( "{\"error\": \"init: %s\"}\n", fdgpu_last_error() ); return 1;
  }
  ulong pub0 = 0UL, pub1 = 0UL;
  int rc = run_batch( vt, mc, dcache, payload, desc, 0UL, &pub0 );
  if( rc || pub0 != N_FRAG ) { printf( "{\"error\": \"warm-up batch rc %d published %lu\"}\n", rc, pub0 ); return 1; }

  int fds[ 16 ]; int n_fds = driver_fds( fds, 16 );
  int allow[ MAX_NR ], n_allow = 0, ioctl_ok = 0;
  if( discover ) {
    /* base set: what the handler itself and the process teardown need */
    char const * base[] = { "rt_sigreturn", "exit", "exit_group" };
    for( unsigned i=0; i<sizeof(base)/sizeof(base[0]); i++ ) { int nr = nr_of( base[i] ); if( nr >= 0 ) allow[ n_allow++ ] = nr; }
  } else {
    for( int i=2; i<argc; i++ ) {
      if( !strcmp( argv[i], "--launcher" ) ) continue;
      if( !strcmp( argv[i], "ioctl" ) ) { ioctl_ok = 1; continue; }
      int nr = nr_of( argv[i] );
      if( nr < 0 ) { printf( "{\"error\": \"unknown syscall %s\"}\n", argv[i] ); return 1; }
      allow[ n_allow++ ] = nr;
    }
  }
  struct sigaction sa; memset( &sa, 0, sizeof(sa) );
  sa.sa_sigaction = on_sigsys; sa.sa_flags = SA_SIGINFO;
  sigaction( SIGSYS, &sa, NULL );
  g_enforce = !discover;
  fflush( stdout ); fflush( stderr );

  /* ---- sandbox ---- */
  rc = install( allow, n_allow, ioctl_ok, fds, n_fds );
  if( rc ) { printf( "{\"error\": \"seccomp install %d (errno %d)\"}\n", rc, errno ); return 1; }

  /* ---- run under the filter ---- */
  ulong t0 = now_ns();
  rc = run_batch( vt, mc, dcache, payload, desc + N_FRAG, N_FRAG, &pub1 );
  ulong dt = now_ns() - t0;

  char extra[ 64 ];
  snprintf( extra, sizeof(extra), "\"launcher\": %d, ", launcher );
  report( "tile", argv[1], rc, N_FRAG, pub1, dt, n_fds, extra );
  /* exit without teardown: the HIP runtime's destructors would make syscalls the policy does not need */
  fdsb_tramp( SYS_exit_group, ( rc || pub1 != N_FRAG ) ? 1 : 0, 0, 0, 0, 0, 0 );
  return 0;
}
