#!/usr/bin/env python3
"""Generate tools/instprobe/instprobe2.hip: VALU issue-rate probe with explicit registers.

Round 2's probe let the compiler place the operands, so VGPR banks (register index mod 4) were
whatever the allocator chose, and every v_mad_u64_u32 wrote vcc.  Here every variant is one inline-asm
loop (no compiler code inside the timed region) over 16 independent chains with the operand banks
chosen on purpose, run at 1, 2, 4 and 8 waves per SIMD:

  *_dist   the sources of each instruction sit in distinct banks
  *_same   the sources share the destination chain's bank
  *_dup    src1 == src2 (one register read twice), bank distinct from the chain
  *_const  inline constants only (one VGPR read per instruction)

The host prints cycles per wave64 instruction per SIMD from the shader clock (s_memtime) of each
block and from the kernel's wall time x the s_memtime / s_memrealtime clock.  The clock is
cross-checked by the GRBM_GUI_ACTIVE / 8 / wall PMC method of MI355X_MICROARCH.md (rocprofv3 pass).
"""
import os

CH = 16          # independent chains per lane
REP = 4          # chain sweeps per loop iteration (64 instructions per iteration)
CHAIN0 = 8       # chain registers v8..v39 (bank = index % 4)
SRC0 = 40        # shared source registers v40..v47: S[b] = v(40+b), S2[b] = v(44+b), bank b
# (all under 64 VGPRs, so 8 waves per SIMD fit)


def reg(i):
    return f"v{i}"


def pair(i):
    return f"v[{i}:{i + 1}]"


def S(b):
    return SRC0 + b % 4


def S2(b):
    return SRC0 + 4 + b % 4


def body(kind):
    """instruction text for one sweep over the chains, and the registers it uses"""
    lines = []
    used = set()
    for c in range(CH):
        if kind.startswith(("mad64", "lshladd64", "pkfma", "lshr64")):
            C = CHAIN0 + 2 * c                                  # pairs in banks {0,1} / {2,3} alternately
            cb = C % 4
            if kind.endswith("_same"):                          # sources in the accumulator's banks
                A, B = S(cb), S(cb + 1)
            else:                                               # the other two banks
                A, B = S(cb + 2), S(cb + 3)
            used |= {C, C + 1, A, B}
            if kind.startswith("mad64"):
                sd = "vcc" if kind.startswith("mad64v") else f"s[{40 + 2 * (c % 8)}:{41 + 2 * (c % 8)}]"
                lines.append(f"v_mad_u64_u32 {pair(C)}, {sd}, {reg(A)}, {reg(B)}, {pair(C)}")
            elif kind.startswith("lshr64"):                     # the field carries (64-bit shift)
                lines.append(f"v_lshrrev_b64 {pair(C)}, 26, {pair(C)}")
            elif kind.startswith("lshladd64"):
                lines.append(f"v_lshl_add_u64 {pair(C)}, {pair(C)}, 1, {pair(min(A, B))}")
            else:                                               # packed f32 FMA on pairs
                lines.append(f"v_pk_fma_f32 {pair(C)}, {pair(C)}, {pair(min(A, B))}, {pair(min(A, B))}")
            continue
        C = CHAIN0 + c
        cb = C % 4
        if kind.endswith("_same"):
            A, B = S(cb), S2(cb)
        elif kind.endswith("_dup"):
            A = B = S(cb + 1)
        else:
            A, B = S(cb + 1), S(cb + 2)
        op = kind.split("_")[0]
        if op == "fma":
            if kind.endswith("_const"):
                lines.append(f"v_fma_f32 {reg(C)}, {reg(C)}, 0.5, 1.0"); used |= {C}
            else:
                lines.append(f"v_fma_f32 {reg(C)}, {reg(C)}, {reg(A)}, {reg(B)}"); used |= {C, A, B}
        elif op == "addf":
            if kind.endswith("_const"):
                lines.append(f"v_add_f32 {reg(C)}, 0.5, {reg(C)}"); used |= {C}
            else:
                lines.append(f"v_add_f32 {reg(C)}, {reg(A)}, {reg(C)}"); used |= {C, A}
        elif op == "add":
            if kind.endswith("_const"):
                lines.append(f"v_add_u32 {reg(C)}, 7, {reg(C)}"); used |= {C}
            else:
                lines.append(f"v_add_u32 {reg(C)}, {reg(A)}, {reg(C)}"); used |= {C, A}
        elif op == "mullo":
            lines.append(f"v_mul_lo_u32 {reg(C)}, {reg(C)}, {reg(A)}"); used |= {C, A}
        elif op == "bitop3":
            lines.append(f"v_bitop3_b32 {reg(C)}, {reg(C)}, {reg(A)}, {reg(B)} bitop3:0x96"); used |= {C, A, B}
        elif op == "mov":
            lines.append(f"v_mov_b32 {reg(C)}, {reg(A)}"); used |= {C, A}
        elif op == "lshr32":
            lines.append(f"v_lshrrev_b32 {reg(C)}, 13, {reg(C)}"); used |= {C}
        elif op == "lshlor":
            lines.append(f"v_lshl_or_b32 {reg(C)}, {reg(C)}, 3, {reg(A)}"); used |= {C, A}
        elif op == "lshladd32":
            lines.append(f"v_lshl_add_u32 {reg(C)}, {reg(C)}, 3, {reg(A)}"); used |= {C, A}
        elif op == "cndmask":
            lines.append(f"v_cndmask_b32 {reg(C)}, {reg(C)}, {reg(A)}, vcc"); used |= {C, A}
        elif op == "addco":
            lines.append(f"v_add_co_u32 {reg(C)}, vcc, {reg(A)}, {reg(C)}"); used |= {C, A}
        elif op == "alignbit":                                  # SHA-512's 64-bit rotations (one half each)
            lines.append(f"v_alignbit_b32 {reg(C)}, {reg(C)}, {reg(A)}, 13"); used |= {C, A}
        elif op == "bfi":                                       # SHA-512's Ch
            lines.append(f"v_bfi_b32 {reg(C)}, {reg(A)}, {reg(C)}, {reg(B)}"); used |= {C, A, B}
        elif op == "perm":                                      # byte swaps of the message words
            lines.append(f"v_perm_b32 {reg(C)}, {reg(C)}, {reg(A)}, {reg(B)}"); used |= {C, A, B}

        else:
            raise ValueError(kind)
    return lines, used


KINDS = ["fma_dist", "fma_same", "fma_dup", "fma_const", "addf_dist", "addf_same", "addf_const",
         "add_dist", "add_same", "add_const", "mullo_dist", "bitop3_dist", "bitop3_same", "mov_dist",
         "pkfma_dist", "pkfma_same", "mad64s_dist", "mad64s_same", "mad64v_dist", "lshladd64_dist",
         "alignbit_dist", "bfi_dist", "perm_dist", "lshr64_dist", "lshr32_dist", "lshlor_dist", "lshladd32_dist",
         "cndmask_dist", "addco_dist"]


def kernel(kind):
    lines, used = body(kind)
    loop = []
    for _ in range(REP):
        loop += lines
    init = [f"v_mov_b32 {reg(r)}, %1" if r % 3 else f"v_add_u32 {reg(r)}, %1, %1" for r in sorted(used)]
    asm = "\\n\\t".join(init + ["s_mov_b32 s20, %0", "1:"] + loop +
                        ["s_sub_u32 s20, s20, 1", "s_cmp_lg_u32 s20, 0", "s_cbranch_scc1 1b"])
    clob = ", ".join(f'"{reg(r)}"' for r in sorted(used))
    sclob = '"s20", "scc", "vcc"' + "".join(f', "s{40 + i}"' for i in range(16))
    per = CH * REP
    return f'''
__global__ void __launch_bounds__( 256 ) k_{kind}( unsigned iters, unsigned seed, unsigned * out, unsigned long long * clk ) {{
  unsigned long long c0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  asm volatile( "{asm}" :: "s"( iters ), "v"( seed + threadIdx.x ) : {clob}, {sclob}, "memory" );
  unsigned long long c1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  if( threadIdx.x == 0 ) {{ unsigned long long * o = clk + 4 * blockIdx.x; o[0] = c0; o[1] = c1; o[2] = r0; o[3] = r1; }}
  if( seed == 0x12345678u ) out[0] = 1u;
}}
static int const per_{kind} = {per};
'''


def main():
    here = os.path.dirname(os.path.abspath(__file__))
    src = ['// GENERATED by gen_instprobe2.py -- do not edit.  See that script for what each variant measures.',
           '// build: hipcc --offload-arch=gfx950 -O3 -o tools/instprobe/instprobe2 tools/instprobe/instprobe2.hip',
           '#include <hip/hip_runtime.h>', '#include <stdio.h>', '#include <stdlib.h>', '#include <algorithm>',
           '#include <vector>']
    for k in KINDS:
        src.append(kernel(k))
    table = ",\n    ".join(f'{{ "{k}", k_{k}, per_{k} }}' for k in KINDS)
    src.append(f'''
typedef void (*kfn)( unsigned, unsigned, unsigned *, unsigned long long * );
int main( int argc, char ** argv ) {{
  struct {{ char const * name; kfn f; int per; }} ks[] = {{
    {table} }};
  unsigned iters = argc > 1 ? (unsigned)atoi( argv[1] ) : 2048u;
  int ncu = 0; hipDeviceGetAttribute( &ncu, hipDeviceAttributeMultiprocessorCount, 0 );
  unsigned * out; hipMalloc( &out, 4 );
  int maxb = ncu * 8;
  unsigned long long * clk; hipMalloc( &clk, (size_t)maxb * 4 * sizeof(unsigned long long) );
  std::vector<unsigned long long> hc( (size_t)maxb * 4 );
  hipEvent_t a, b; hipEventCreate( &a ); hipEventCreate( &b );
  /* warm the clock up: 2 s of back-to-back launches (MI355X_MICROARCH.md DVFS item 6) */
  {{ hipEventRecord( a ); float ms = 0.f;
     while( ms < 2000.f ) {{ for( int i=0; i<20; i++ ) hipLaunchKernelGGL( k_fma_dist, dim3(maxb), dim3(256), 0, 0, iters, 1u, out, clk );
       hipEventRecord( b ); hipEventSynchronize( b ); hipEventElapsedTime( &ms, a, b ); }} }}
  printf( "%-16s %5s %9s %9s %10s %10s %10s\\n", "variant", "w/SIMD", "wall_ms", "clk_MHz", "cyc_blk", "cyc_wall", "Tlaneop/s" );
  for( auto & k : ks ) for( int w : {{ 1, 2, 4, 8 }} ) {{
    int blocks = ncu * w;                         /* 256-thread blocks: w blocks per CU = w waves per SIMD */
    hipLaunchKernelGGL( k.f, dim3(blocks), dim3(256), 0, 0, 8u, 1u, out, clk );
    float best = 1e30f; double cyc_blk = 0., mhz = 0.;
    for( int r=0; r<5; r++ ) {{
      hipEventRecord( a ); hipLaunchKernelGGL( k.f, dim3(blocks), dim3(256), 0, 0, iters, 1u, out, clk ); hipEventRecord( b );
      hipEventSynchronize( b ); float ms; hipEventElapsedTime( &ms, a, b );
      if( ms < best ) {{
        best = ms;
        hipMemcpy( hc.data(), clk, (size_t)blocks * 4 * sizeof(unsigned long long), hipMemcpyDeviceToHost );
        std::vector<double> dc( blocks ); double sc = 0., sr = 0.;
        for( int i=0; i<blocks; i++ ) {{ dc[i] = (double)( hc[4*i+1] - hc[4*i] ); sc += dc[i]; sr += (double)( hc[4*i+3] - hc[4*i+2] ); }}
        std::sort( dc.begin(), dc.end() );
        mhz = sr > 0. ? sc / sr * 100. : 0.;        /* s_memrealtime ticks at 100 MHz */
        cyc_blk = dc[ blocks / 2 ];                  /* median block: its wave's own cycles, start to end */
      }}
    }}
    double n = (double)iters * k.per;             /* wave-instructions per wave */
    double cb = cyc_blk / ( n * w );               /* w co-resident waves share the SIMD over that interval */
    double cw = mhz * 1e3 * best / ( n * w );      /* wall x clock */
    double rate = (double)blocks * 256.0 * n / ( best * 1e-3 ) * 1e-12;
    printf( "%-16s %5d %9.3f %9.0f %10.2f %10.2f %10.2f\\n", k.name, w, best, mhz, cb, cw, rate );
  }}
  return 0;
}}
''')
    with open(os.path.join(here, "instprobe2.hip"), "w") as f:
        f.write("\n".join(src))


if __name__ == "__main__":
    main()
