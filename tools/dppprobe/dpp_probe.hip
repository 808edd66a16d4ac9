// Probe: VOP2 DPP arithmetic semantics on gfx950 (v_add/v_sub/v_subrev _u32 with quad_perm).
#include <hip/hip_runtime.h>
#include <cstdio>
typedef unsigned u32;
#define OP(name, PERM) \
  asm volatile( "s_nop 1\n\t" name "_dpp %0, %1, %2 " PERM " row_mask:0xf bank_mask:0xf\n\t" : "=&v"(r) : "v"(a), "v"(b) )
__global__ void k( u32 * out ) {
  u32 l = threadIdx.x;
  u32 a = l * 1000u + 7u, b = l * 3u + 1u, r;
  OP( "v_add_u32", "quad_perm:[0,0,0,0]" );    out[l*6+0] = r;
  OP( "v_sub_u32", "quad_perm:[3,3,3,3]" );    out[l*6+1] = r;
  OP( "v_subrev_u32", "quad_perm:[1,1,1,1]" ); out[l*6+2] = r;
  OP( "v_add_u32", "quad_perm:[2,2,2,2]" );    out[l*6+3] = r;
  u32 x;
  asm volatile( "s_nop 1\n\tv_mov_b32_dpp %0, %1 quad_perm:[2,2,2,2] row_mask:0xf bank_mask:0xf\n\t" : "=&v"(x) : "v"(a) );
  out[l*6+4] = x + b;
  out[l*6+5] = 0;
}
int main() {
  u32 * d; hipMalloc( &d, 64*6*4 ); hipMemset( d, 0, 64*6*4 );
  hipLaunchKernelGGL( k, dim3(1), dim3(64), 0, 0, d );
  u32 h[64*6]; hipMemcpy( h, d, sizeof(h), hipMemcpyDeviceToHost );
  int bad = 0;
  for( u32 l=0; l<64; l++ ) {
    u32 q = l & ~3u;
    u32 A = [&](u32 s){ return s*1000u+7u; }(0), b = l*3u+1u;
    (void)A;
    u32 e[5] = { (q+0)*1000u+7u + b, (q+3)*1000u+7u - b, b - ((q+1)*1000u+7u), (q+2)*1000u+7u + b, (q+2)*1000u+7u + b };
    for( int i=0; i<5; i++ ) if( h[l*6+i] != e[i] ) { if( bad < 20 ) printf( "lane %u op %d got %u want %u\n", l, i, h[l*6+i], e[i] ); bad++; }
  }
  printf( "dpp probe: %s (%d mismatches)\n", bad ? "FAIL" : "ok", bad );
  return bad ? 1 : 0;
}
