/* Host timing-call cost on the box: clock_gettime(CLOCK_MONOTONIC) and rdtsc, ns per call.
   build: gcc -O2 -o tools/hostprobe/clock_cost tools/hostprobe/clock_cost.c */
#include <stdio.h>
#include <time.h>
#include <x86intrin.h>
static unsigned long now_ns( void ) { struct timespec ts; clock_gettime( CLOCK_MONOTONIC, &ts ); return (unsigned long)ts.tv_sec * 1000000000UL + (unsigned long)ts.tv_nsec; }
int main( void ) {
  unsigned long n = 2000000, s = 0, t0 = now_ns();
  for( unsigned long i=0; i<n; i++ ) s += now_ns();
  unsigned long t1 = now_ns();
  unsigned long c0 = __rdtsc();
  for( unsigned long i=0; i<n; i++ ) s += __rdtsc();
  unsigned long c1 = __rdtsc(), t2 = now_ns();
  printf( "clock_gettime %.1f ns/call  rdtsc %.1f ns/call  tsc %.3f GHz  (%lu)\n", (double)( t1 - t0 ) / n,
          (double)( t2 - t1 ) / n, (double)( c1 - c0 ) / (double)( t2 - t1 ), s & 1 );
  return 0;
}
