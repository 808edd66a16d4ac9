#!/bin/bash
# Round 4's GPU jobs, one parameterised runner (replaces the one-off tools/gpu_r04_*.sh scripts).
#   usage: gpurun --timeout 900 -- 'bash tools/r04_jobs.sh <job>'
# Every job writes under gpurun_out/r04<x>/ (the letter in the table) and is copied into profiles/r04/<x>/.
# Arms of an A/B run interleaved on one box (ABBA or ABC..CBA); each step has its own time limit (gpu_job.sh).
#
#   job          dir  what
#   huge_ab      g    THP link / 4 records per gather group / --stream-first / max_uncopied / copy wait
#   hwq_ab       h    GPU_MAX_HW_QUEUES of the tile processes, 2 paced tiles, 3 max tiles, pinning
#   thp_ab       i    THP link, 4 records per gather group, 32 gather CUs (quiet box)
#   cus_ab       j    which 16 CUs the gathers get; new defaults through the vtile GPU tests
#   latctx_ab    k    engine contexts per paced tile (1 / 2 / 3)
#   split_ab     m    disjoint CU halves per context (+ kernel traces)
#   childprof    n    kernel traces of the paced tile process at 10M frags/s
#   excl_ab      o    latency-path workgroups alone on their CU (+ latency8x parity tests)
#   excl2_ab     p    exclusivity variants (two per CU, walk only, prep only)
#   excl3_ab     q    exclusivity repeat at the default paced rates
#   cw_ab        r    bigger gathers on the max legs (copy wait / uncopied bound)
#   tput_ab      s    gather size of the max legs: 50 us / 200 us / 500 us / 1 ms
#   rehearse     t    N=2 (torchrun) and N=4 (self-launch) on one GPU
#   lt2_ab       u    1 vs 2 paced tiles with exclusivity
#   gprobe_pmc   v    fabric request sizes of tools/gatherprobe
#   clock_ab     w    one clock read per tile-loop pass (needs firedancer_amd/ab_vtile_old.so)
#   memtype      x    tools/gatherprobe/gather_memtype: host memory types of the in / out regions
#   copy_ab      y    host-copy intake vs zero-copy at 2 / 3 / 4 tiles
#   t3_ab        z    2 vs 3 vs 4 tiles at the final defaults
#   gsize_ab     gs   max-leg gathers of 4K / 16K / 32K / 64K records (copy_min with copy wait and uncopied bound)
#   big_ab       gt   with ~20K-record gathers (the new max-leg default): 2 vs 3 tiles, 2 producers
#   host_ab      ha   tile host trims (one tcache probe per verdict, one fault check per frag) vs the previous
#                     build (firedancer_amd/ab_vtile_old.so)
#   pf_ab        pf   tile-loop prefetch distance 1 / 2 / 4 / 8 own frags, now that the loop bounds the max rate
#   o3_ab        o3   the tile library at -O3 -march=x86-64-v3 (firedancer_amd/ab_vtile_o3.so) vs -O2
#   first_ab     fi   stream legs before the bench process opens its own GPU queues (--stream-first): the paced
#                     legs' occasional 0.5-1.7 ms gather-start stalls
#   pcw_ab       pcw  the paced tile's copy wait (25 / 50 / 100 / 200 us): gather launches are ~12 % of its loop
#                     (run with --stream-copy-wait-us, which then covered the paced legs)
#   pcw2_ab      pcw2 paced copy wait 25 (the new bench default) vs 12.5 us
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp

# run_arms <outdir> <common bench args> <name>=<extra args> ... : one gpu_job.sh step per arm
run_arms() {
  local out="$1" common="$2"; shift 2
  mkdir -p "gpurun_out/$out"
  local steps=() a name extra env
  for a in "$@"; do
    name="${a%%=*}"; extra="${a#*=}"; env=""
    case "$extra" in ENV:*) env="${extra#ENV:}"; env="${env%%;*}"; extra="${extra#*;}";; esac
    steps+=( "$name:200:$env python3 bench.py $common $extra --detail-out gpurun_out/$out/$name.json > gpurun_out/$out/$name.out" )
  done
  bash tools/gpu_job.sh "${steps[@]}"
}

# Arms use today's flags. A job run before a default changed pins the setting it ran with:
#   R3   = round 3's gather setup (link in 4 KiB pages, 1 record per gather group), the base of g / h / i;
#   EARLY = the stream defaults before jobs q and s (latency-path workgroups not exclusive, max legs copying
#           like the paced legs), for jobs g .. p.
R3="--stream-no-huge --stream-gather-rpb 1"
EARLY="--stream-cu-exclusive -1 --stream-tput-copy-wait-us 0 --stream-tput-max-uncopied 0"
VT="vt:400:python -u -m pytest tests/test_gpu_vtile.py tests/test_gpu_faults.py tests/test_gpu_stream_parity.py -x -q --timeout 200 --timeout-method thread"
Q="--steps 2 --warmup 1 --txns 262144 --no-cpu-baseline --no-extra-configs --latency-batch 0"
CHILD="python3 bench.py --stream-child --stream-device 0 --stream-proc 0 --stream-procs 1 --stream-token pp --stream-seed 1234 --txns 65536 --stream-rates 10e6 --stream-only-paced --stream-paced-seconds 2"

case "$1" in
huge_ab)
  bash tools/gpu_job.sh "$VT" &&
  run_arms r04g "$Q $EARLY --stream-rates 5e6,10e6 --stream-paced-seconds 2 --stream-seconds 5 --stream-unrel-seconds 1 --stream-prof" \
    "base1=$R3" "cw200a=$R3 --stream-copy-wait-us 200 --stream-max-uncopied 65536" "rpb4a=--stream-no-huge" \
    "huge1=--stream-gather-rpb 1" "first1=$R3 --stream-first" "unc64a=$R3 --stream-max-uncopied 65536" \
    "unc64b=$R3 --stream-max-uncopied 65536" "first2=$R3 --stream-first" "huge2=--stream-gather-rpb 1" "rpb4b=--stream-no-huge" \
    "cw200b=$R3 --stream-copy-wait-us 200 --stream-max-uncopied 65536" "base2=$R3" ;;
hwq_ab)
  bash tools/gpu_job.sh "$VT" &&
  run_arms r04h "$Q $EARLY $R3 --stream-rates 7.5e6,10e6,12.5e6 --stream-paced-seconds 2 --stream-seconds 5 --stream-unrel-seconds 1 --stream-prof" \
    base1= "q8a=--stream-hw-queues 8" "lt2a=--stream-lat-tiles 2" "lt2q8a=--stream-lat-tiles 2 --stream-hw-queues 8" \
    "t3q12a=--stream-tiles 3 --stream-hw-queues 12" "low1=ENV:FDGPU_LINK_PIN=lowest;" "low2=ENV:FDGPU_LINK_PIN=lowest;" \
    "t3q12b=--stream-tiles 3 --stream-hw-queues 12" "lt2q8b=--stream-lat-tiles 2 --stream-hw-queues 8" \
    "lt2b=--stream-lat-tiles 2" "q8b=--stream-hw-queues 8" base2= ;;
thp_ab)
  mkdir -p gpurun_out/r04i
  (cat /sys/kernel/mm/transparent_hugepage/enabled /sys/devices/system/clocksource/clocksource0/current_clocksource
   for g in /sys/kernel/iommu_groups/*; do cat $g/type 2>/dev/null; done | sort | uniq -c) > gpurun_out/r04i/sysinfo.txt 2>&1
  run_arms r04i "$Q $EARLY --stream-rates 7.5e6,10e6 --stream-paced-seconds 2 --stream-seconds 5 --stream-unrel-seconds 1 --stream-prof" \
    "base1=$R3" "huge1=--stream-gather-rpb 1" "rpb4a=--stream-no-huge" "cu32a=$R3 --stream-gather-cus 32" hr4a= hr4b= \
    "cu32b=$R3 --stream-gather-cus 32" "rpb4b=--stream-no-huge" "huge2=--stream-gather-rpb 1" "base2=$R3" ;;
cus_ab)
  bash tools/gpu_job.sh "$VT" &&
  run_arms r04j "$Q $EARLY --stream-rates 7.5e6,10e6 --stream-paced-seconds 2 --stream-seconds 5 --stream-unrel-seconds 1 --stream-prof" \
    base1= "spr1a=--stream-gather-cu-spread 1" "first1a=--stream-gather-cu-spread 2" \
    "r3a=--stream-no-huge --stream-gather-rpb 1" "r3b=--stream-no-huge --stream-gather-rpb 1" \
    "first1b=--stream-gather-cu-spread 2" "spr1b=--stream-gather-cu-spread 1" base2= ;;
latctx_ab)
  run_arms r04k "$Q $EARLY --stream-rates 5e6,7.5e6,10e6,12.5e6 --stream-paced-seconds 2 --stream-seconds 3 --stream-unrel-seconds 1 --stream-prof" \
    c2a= "c1a=--stream-lat-ctx 1" "c3a=--stream-lat-ctx 3" "c3b=--stream-lat-ctx 3" "c1b=--stream-lat-ctx 1" c2b= ;;
split_ab)
  P="$Q $EARLY --steps 1 --warmup 0 --txns 65536 --stream-rates 10e6 --stream-only-paced --stream-paced-seconds 2"
  mkdir -p gpurun_out/r04m
  bash tools/gpu_job.sh \
    "splitt:300:python -u -m pytest tests/test_gpu_vtile.py -k 'cu_split or stream_run_link' -x -q --timeout 200 --timeout-method thread" \
    "pprof0:200:rocprofv3 --kernel-trace --stats -d gpurun_out/r04m/prof0 -o run -- python3 bench.py $P --detail-out gpurun_out/r04m/pprof0.json > gpurun_out/r04m/pprof0.out" \
    "pprof1:200:rocprofv3 --kernel-trace --stats -d gpurun_out/r04m/prof1 -o run -- python3 bench.py $P --stream-lat-cu-split 1 --detail-out gpurun_out/r04m/pprof1.json > gpurun_out/r04m/pprof1.out" &&
  run_arms r04m "$Q $EARLY --stream-rates 5e6,7.5e6,10e6,12.5e6 --stream-paced-seconds 2 --stream-seconds 3 --stream-unrel-seconds 1 --stream-prof" \
    s0a= "s1a=--stream-lat-cu-split 1" "s1b=--stream-lat-cu-split 1" s0b= ;;
childprof)
  mkdir -p gpurun_out/r04n
  bash tools/gpu_job.sh \
    "cp0:200:rocprofv3 --kernel-trace --stats -d gpurun_out/r04n/c2 -o run -- $CHILD --stream-cu-exclusive -1 > gpurun_out/r04n/c2.out" \
    "cp1:200:rocprofv3 --kernel-trace --stats -d gpurun_out/r04n/c2split -o run -- $CHILD --stream-cu-exclusive -1 --stream-lat-cu-split 1 > gpurun_out/r04n/c2split.out" \
    "cp2:200:rocprofv3 --kernel-trace --stats -d gpurun_out/r04n/c1 -o run -- $CHILD --stream-cu-exclusive -1 --stream-lat-ctx 1 > gpurun_out/r04n/c1.out" ;;
excl_ab)
  mkdir -p gpurun_out/r04o
  bash tools/gpu_job.sh \
    "xtests:400:python -u -m pytest tests -m gpu -k 'latency8x or cu_split' -x -q --timeout 200 --timeout-method thread" \
    "xprof:200:rocprofv3 --kernel-trace --stats -d gpurun_out/r04o/cx -o run -- $CHILD --stream-cu-exclusive 1 > gpurun_out/r04o/cx.out" &&
  run_arms r04o "$Q --stream-tput-copy-wait-us 0 --stream-tput-max-uncopied 0 --stream-rates 5e6,7.5e6,10e6,12.5e6 --stream-paced-seconds 2 --stream-seconds 3 --stream-unrel-seconds 1 --stream-prof" \
    "e0a=--stream-cu-exclusive -1" "e1a=--stream-cu-exclusive 1" "e1b=--stream-cu-exclusive 1" "e0b=--stream-cu-exclusive -1" ;;
excl2_ab)
  run_arms r04p "$Q --stream-tput-copy-wait-us 0 --stream-tput-max-uncopied 0 --stream-rates 2e6,5e6,7.5e6,10e6,12.5e6 --stream-paced-seconds 2 --stream-seconds 3 --stream-unrel-seconds 1" \
    "x0a=--stream-cu-exclusive -1" "x1a=--stream-cu-exclusive 1" "x2a=--stream-cu-exclusive 2" "x3a=--stream-cu-exclusive 3" \
    "x4a=--stream-cu-exclusive 4" "x4b=--stream-cu-exclusive 4" "x3b=--stream-cu-exclusive 3" "x2b=--stream-cu-exclusive 2" \
    "x1b=--stream-cu-exclusive 1" "x0b=--stream-cu-exclusive -1" ;;
excl3_ab)
  run_arms r04q "$Q --stream-tput-copy-wait-us 0 --stream-tput-max-uncopied 0 --stream-paced-seconds 2 --stream-seconds 3 --stream-unrel-seconds 1" \
    "y0a=--stream-cu-exclusive -1" "y1a=--stream-cu-exclusive 1" "y1b=--stream-cu-exclusive 1" "y0b=--stream-cu-exclusive -1" \
    "y0c=--stream-cu-exclusive -1" "y1c=--stream-cu-exclusive 1" ;;
cw_ab)
  run_arms r04r "$Q --stream-rates 10e6 --stream-paced-seconds 2 --stream-seconds 5 --stream-unrel-seconds 1 --stream-prof" \
    "b1=--stream-tput-copy-wait-us 0 --stream-tput-max-uncopied 0" \
    "w100a=--stream-tput-copy-wait-us 100 --stream-tput-max-uncopied 32768" \
    "w200a=--stream-tput-copy-wait-us 200 --stream-tput-max-uncopied 65536" \
    "u32a=--stream-tput-copy-wait-us 0 --stream-tput-max-uncopied 32768" \
    "u32b=--stream-tput-copy-wait-us 0 --stream-tput-max-uncopied 32768" \
    "w200b=--stream-tput-copy-wait-us 200 --stream-tput-max-uncopied 65536" \
    "w100b=--stream-tput-copy-wait-us 100 --stream-tput-max-uncopied 32768" \
    "b2=--stream-tput-copy-wait-us 0 --stream-tput-max-uncopied 0" ;;
tput_ab)
  run_arms r04s "$Q --stream-rates 10e6 --stream-paced-seconds 2 --stream-seconds 5 --stream-unrel-seconds 1 --stream-prof" \
    "old1=--stream-tput-copy-wait-us 0 --stream-tput-max-uncopied 0" d1= \
    "w500a=--stream-tput-copy-wait-us 500 --stream-tput-max-uncopied 131072" \
    "w1ka=--stream-tput-copy-wait-us 1000 --stream-tput-max-uncopied 131072" \
    "w1kb=--stream-tput-copy-wait-us 1000 --stream-tput-max-uncopied 131072" \
    "w500b=--stream-tput-copy-wait-us 500 --stream-tput-max-uncopied 131072" d2= \
    "old2=--stream-tput-copy-wait-us 0 --stream-tput-max-uncopied 0" ;;
rehearse)
  mkdir -p gpurun_out/r04t
  bash tools/gpu_job.sh \
    "n2:400:bash tools/rehearse_n2.sh --stream-rates 2e6,4e6 --stream-paced-seconds 2 --detail-out gpurun_out/r04t/n2.json > gpurun_out/r04t/n2.out" \
    "n4:400:FDGPU_BENCH_ONE_DEVICE=1 python3 bench.py --gpus 4 $Q --steps 3 --stream-rates 1e6,2e6 --stream-paced-seconds 2 --stream-seconds 3 --stream-unrel-seconds 1 --detail-out gpurun_out/r04t/n4.json > gpurun_out/r04t/n4.out" ;;
lt2_ab)
  run_arms r04u "$Q --stream-rates 7.5e6,10e6,12.5e6,15e6 --stream-paced-seconds 2 --stream-seconds 3 --stream-unrel-seconds 1" \
    t1a= "t2a=--stream-lat-tiles 2" "t2c1a=--stream-lat-tiles 2 --stream-lat-ctx 1" \
    "t2c1b=--stream-lat-tiles 2 --stream-lat-ctx 1" "t2b=--stream-lat-tiles 2" t1b= ;;
gprobe_pmc)
  mkdir -p gpurun_out/r04v
  bash tools/gpu_job.sh \
    "gp:120:tools/gatherprobe/gather_probe > gpurun_out/r04v/probe.log" \
    "gpr:90:timeout -s KILL 60 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum -f csv -d gpurun_out/r04v/rd -o run -- tools/gatherprobe/gather_probe" \
    "gpw:90:timeout -s KILL 60 rocprofv3 --pmc TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum -f csv -d gpurun_out/r04v/wr -o run -- tools/gatherprobe/gather_probe" ;;
clock_ab)
  run_arms r04w "$Q --stream-rates 7.5e6,10e6,12.5e6,15e6 --stream-paced-seconds 2 --stream-seconds 4 --stream-unrel-seconds 1" \
    new1= "old1=ENV:FDGPU_VTILE_LIB=firedancer_amd/ab_vtile_old.so;" "old2=ENV:FDGPU_VTILE_LIB=firedancer_amd/ab_vtile_old.so;" new2= ;;
memtype)
  mkdir -p gpurun_out/r04x
  bash tools/gpu_job.sh "mt:240:tools/gatherprobe/gather_memtype > gpurun_out/r04x/memtype.log" ;;
copy_ab)
  run_arms r04y "$Q --stream-rates 5e6 --stream-paced-seconds 1 --stream-seconds 4 --stream-unrel-seconds 1 --stream-prof" \
    zc2= cp2=--stream-copy "cp3=--stream-copy --stream-tiles 3" "cp4=--stream-copy --stream-tiles 4" "zc3=--stream-tiles 3" ;;
t3_ab)
  run_arms r04z "$Q --stream-rates 5e6 --stream-paced-seconds 1 --stream-seconds 5 --stream-unrel-seconds 1 --stream-prof" \
    t2a= "t3a=--stream-tiles 3" "t3b=--stream-tiles 3" t2b= t2c= "t3c=--stream-tiles 3" \
    "t4a=--stream-tiles 4 --stream-producers 2" "t3p2=--stream-tiles 3 --stream-producers 2" ;;
gsize_ab)
  G16="--stream-tput-copy-wait-us 1000 --stream-tput-copy-min 16384 --stream-tput-max-uncopied 131072"
  G32="--stream-tput-copy-wait-us 2000 --stream-tput-copy-min 32768 --stream-tput-max-uncopied 131072"
  G64="--stream-tput-copy-wait-us 4000 --stream-tput-copy-min 65536 --stream-tput-max-uncopied 262144"
  run_arms r04gs "$Q --stream-tput-copy-wait-us 200 --stream-tput-copy-min 0 --stream-tput-max-uncopied 65536 --stream-rates 5e6 --stream-paced-seconds 1 --stream-seconds 5 --stream-unrel-seconds 1 --stream-prof" \
    d1= "g16a=$G16" "g32a=$G32" "g64a=$G64" "g64b=$G64" "g32b=$G32" "g16b=$G16" d2= ;;
big_ab)
  run_arms r04gt "$Q --stream-rates 5e6 --stream-paced-seconds 1 --stream-seconds 5 --stream-unrel-seconds 1 --stream-prof" \
    t2a= "t3a=--stream-tiles 3" "t2p2a=--stream-producers 2" "t2p2b=--stream-producers 2" "t3b=--stream-tiles 3" t2b= ;;
host_ab)
  run_arms r04ha "$Q --stream-rates 10e6 --stream-paced-seconds 2 --stream-seconds 5 --stream-unrel-seconds 1 --stream-prof" \
    new1= "old1=ENV:FDGPU_VTILE_LIB=firedancer_amd/ab_vtile_old.so;" "old2=ENV:FDGPU_VTILE_LIB=firedancer_amd/ab_vtile_old.so;" \
    new2= new3= "old3=ENV:FDGPU_VTILE_LIB=firedancer_amd/ab_vtile_old.so;" ;;
pf_ab)
  run_arms r04pf "$Q --stream-rates 10e6 --stream-paced-seconds 2 --stream-seconds 5 --stream-unrel-seconds 1 --stream-prof" \
    p1a= "p4a=--stream-pf-dist 4" "p8a=--stream-pf-dist 8" "p2a=--stream-pf-dist 2" \
    "p2b=--stream-pf-dist 2" "p8b=--stream-pf-dist 8" "p4b=--stream-pf-dist 4" p1b= ;;
o3_ab)
  run_arms r04o3 "$Q --stream-rates 10e6 --stream-paced-seconds 2 --stream-seconds 5 --stream-unrel-seconds 1 --stream-prof" \
    o2a= "o3a=ENV:FDGPU_VTILE_LIB=firedancer_amd/ab_vtile_o3.so;" "o3b=ENV:FDGPU_VTILE_LIB=firedancer_amd/ab_vtile_o3.so;" \
    o2b= o2c= "o3c=ENV:FDGPU_VTILE_LIB=firedancer_amd/ab_vtile_o3.so;" ;;
first_ab)
  run_arms r04fi "$Q --stream-rates 5e6,10e6 --stream-paced-seconds 3 --stream-seconds 3 --stream-unrel-seconds 1" \
    b1= f1=--stream-first f2=--stream-first b2= b3= f3=--stream-first ;;
pcw_ab)
  run_arms r04pcw "$Q --stream-lat-copy-wait-us 50 --stream-rates 7.5e6,10e6,12.5e6 --stream-paced-seconds 3 --stream-seconds 3 --stream-unrel-seconds 1" \
    c50a= "c100a=--stream-lat-copy-wait-us 100" "c200a=--stream-lat-copy-wait-us 200" "c25a=--stream-lat-copy-wait-us 25" \
    "c25b=--stream-lat-copy-wait-us 25" "c200b=--stream-lat-copy-wait-us 200" "c100b=--stream-lat-copy-wait-us 100" c50b= ;;
pcw2_ab)
  run_arms r04pcw2 "$Q --stream-rates 5e6,7.5e6,10e6,12.5e6 --stream-paced-seconds 3 --stream-seconds 3 --stream-unrel-seconds 1" \
    c25a= "c12a=--stream-lat-copy-wait-us 12.5" "c12b=--stream-lat-copy-wait-us 12.5" c25b= c25c= "c12c=--stream-lat-copy-wait-us 12.5" ;;
*)
  sed -n '2,35p' "$0"; exit 2 ;;
esac
