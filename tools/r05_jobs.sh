#!/bin/bash
# Round-5 GPU jobs: tools/r05_jobs.sh <job>   (each step under its own time limit via tools/gpu_job.sh)
#   pp     : prep role lengths of latency-path batches (FD_PREP_PROBE variant build/ab/pp.so,
#            tools/prep_probe.py) at 1,000 / 2,800 / 8,192 txns, the chain's kernel trace at 2,800 txns,
#            the paced stream parity tests and the launch-thread tests, then an interleaved A/B of the
#            paced legs' launch thread (--stream-lat-launcher 0 / 1)
#   hc     : host copy threads: their parity tests, then max-rate arms with 0 / 1 / 2 copy threads per tile on
#            2, 3 and 4 tiles
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
job="$1"; shift
Q="--steps 2 --warmup 1 --txns 262144 --no-cpu-baseline --no-extra-configs --latency-batch 0"

# run_arms <outdir> <common bench args> <name>=<extra args> ... : one gpu_job.sh step per arm
run_arms() {
  local out="$1" common="$2"; shift 2
  mkdir -p "gpurun_out/$out"
  local steps=() a name extra
  for a in "$@"; do
    name="${a%%=*}"; extra="${a#*=}"
    steps+=( "$name:240:python3 bench.py $common $extra --detail-out gpurun_out/$out/$name.json > gpurun_out/$out/$name.out" )
  done
  bash tools/gpu_job.sh "${steps[@]}"
}

case "$job" in
  tc)
    # kernel trace of one paced leg at 10M frags/s (the stream child alone, under rocprofv3): the batch chain's
    # kernels and the dispatch gaps between them (tools/trace_chain.py)
    d=gpurun_out/r05_tc; mkdir -p $d
    bash tools/gpu_job.sh \
      "ktrace:300:rocprofv3 --kernel-trace -f csv -d $d/t -o run -- python bench.py --stream-child --stream-token tc --stream-procs 1 --stream-only-paced --stream-rates 10e6 --stream-paced-seconds 2 > $d/legs.json" \
      "reduce:200:python tools/trace_chain.py $d > $d/chain.json && rm -rf $d/t"
    ;;
  db)
    # default bench runs of the final build (the driver's command), each with its detail record
    mkdir -p gpurun_out/r05_db
    bash tools/gpu_job.sh \
      "b1:300:python bench.py --detail-out gpurun_out/r05_db/b1.json > gpurun_out/r05_db/b1.line" \
      "b2:300:python bench.py --detail-out gpurun_out/r05_db/b2.json > gpurun_out/r05_db/b2.line" \
      "b3:300:python bench.py --detail-out gpurun_out/r05_db/b3.json > gpurun_out/r05_db/b3.line"
    ;;
  ma)
    # the -A / -R table's additions in affine form (FD_ATAB_MADD=1, now the default) vs the cached form
    # (build/ab/cadd.so): engine-path parity tests, then interleaved headline runs and a kernel trace of each
    d=gpurun_out/r05_ma; mkdir -p $d
    H="python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --latency-batch 0 --stream-frags 0 --no-extra-configs"
    bash tools/gpu_job.sh \
      "tests:900:python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_edges.py tests/test_gpu_hs_top.py tests/test_gpu_torsion.py -q -rA --timeout 300 --timeout-method thread" \
      "m1:200:$H --detail-out $d/m1.json > $d/m1.out" \
      "c1:200:FDGPU_LIB=build/ab/cadd.so $H --detail-out $d/c1.json > $d/c1.out" \
      "m2:200:$H --detail-out $d/m2.json > $d/m2.out" \
      "c2:200:FDGPU_LIB=build/ab/cadd.so $H --detail-out $d/c2.json > $d/c2.out" \
      "m3:200:$H --detail-out $d/m3.json > $d/m3.out" \
      "c3:200:FDGPU_LIB=build/ab/cadd.so $H --detail-out $d/c3.json > $d/c3.out" \
      "km:200:rocprofv3 --kernel-trace --stats -f csv -d $d/km -o run -- $H > $d/km.out" \
      "kc:200:FDGPU_LIB=build/ab/cadd.so rocprofv3 --kernel-trace --stats -f csv -d $d/kc -o run -- $H > $d/kc.out" \
      "lm:200:python tools/latency_probe.py 1024 2800 8192 > $d/lm.out" \
      "lc:200:FDGPU_LIB=build/ab/cadd.so python tools/latency_probe.py 1024 2800 8192 > $d/lc.out"
    ;;
  pz)
    # GPU pauses without this repository's engine, tile or PyTorch: tools/pauseprobe (plain HIP, a one-wave
    # kernel every 50 us, its launch -> start delay) idle and under load, around a paced-only bench run
    d=gpurun_out/r05_pz; mkdir -p $d
    bash tools/gpu_job.sh \
      "pi1:60:tools/pauseprobe/pause_probe i 10 50 > $d/pi1.json" \
      "pb1:60:tools/pauseprobe/pause_probe b 10 50 > $d/pb1.json" \
      "paced:240:python3 bench.py $Q --stream-only-paced --stream-rates 5e6,7.5e6,10e6 --stream-paced-seconds 5 --detail-out $d/paced.json > $d/paced.out" \
      "pb2:60:tools/pauseprobe/pause_probe b 10 50 > $d/pb2.json" \
      "pi2:60:tools/pauseprobe/pause_probe i 10 50 > $d/pi2.json"
    ;;
  pin)
    # the link's CPU choice (an L3 group with room for the producer and the tiles) and the producer / tile
    # placement in each leg: the stream / tile parity tests, then two default bench runs
    mkdir -p gpurun_out/r05_pin
    bash tools/gpu_job.sh \
      "tests:900:python -u -m pytest tests/test_gpu_stream_parity.py tests/test_gpu_stem.py tests/test_gpu_vtile.py -q -rA --timeout 300 --timeout-method thread" \
      "b1:300:FDGPU_LINK_VERBOSE=1 python bench.py --detail-out gpurun_out/r05_pin/b1.json > gpurun_out/r05_pin/b1.line" \
      "b2:300:python bench.py --detail-out gpurun_out/r05_pin/b2.json > gpurun_out/r05_pin/b2.line"
    ;;
  db2|db3)
    # default bench runs of the last engine build (db2: slow list in the walk kernels; db3: the final build),
    # each with its detail record
    o=gpurun_out/r05_$job; mkdir -p $o
    bash tools/gpu_job.sh \
      "b1:300:python bench.py --detail-out $o/b1.json > $o/b1.line" \
      "b2:300:python bench.py --detail-out $o/b2.json > $o/b2.line" \
      "b3:300:python bench.py --detail-out $o/b3.json > $o/b3.line"
    ;;
  pl)
    # the GPU pause log per paced leg (episodes: start ms, longest hold us, copies), default settings
    run_arms r05_pl "$Q --stream-only-paced --stream-rates 2e6,5e6,7.5e6,10e6 --stream-paced-seconds 5" "l1=" "l2=" "l3="
    ;;
  pt)
    # paced tiles: 1 tile x 2 contexts (default) / 2 tiles x 1 context / 2 tiles x 2 contexts (each walk in 1/4)
    run_arms r05_pt "$Q --stream-only-paced --stream-rates 5e6,7.5e6,10e6,12.5e6 --stream-paced-seconds 3" \
      "a1=" "b1=--stream-lat-tiles 2 --stream-lat-ctx 1" "c1=--stream-lat-tiles 2 --stream-lat-share 4" \
      "a2=" "b2=--stream-lat-tiles 2 --stream-lat-ctx 1" "c2=--stream-lat-tiles 2 --stream-lat-share 4"
    ;;
  sf)
    # GPU pauses in the paced legs (paced_gpu_pauses_over_250us) with the bench process's own GPU context open
    # (default: headline first) or not yet (--stream-first: the tile processes run before it touches the GPU)
    run_arms r05_sf "$Q --stream-only-paced --stream-rates 5e6,7.5e6,10e6,12.5e6 --stream-paced-seconds 3" \
      "d1=" "f1=--stream-first" "d2=" "f2=--stream-first" "d3=" "f3=--stream-first"
    ;;
  qs)
    # the latency path's hash role on a quad of lanes (fd_sha512_RAM_quad): the engine-path parity tests (every
    # latency path; latency4s keeps the one-lane role), prep role lengths quad vs one lane (FD_PREP_PROBE build
    # build/ab/pp.so: tools/ab_build.sh pp -DFD_PREP_PROBE=1), then paced arms
    d="gpurun_out/r05_qs"; mkdir -p "$d"
    bash tools/gpu_job.sh \
      "tests:900:python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_hs_top.py tests/test_gpu_edges.py tests/test_gpu_torsion.py tests/test_gpu_callers.py tests/test_gpu_txn.py tests/test_gpu_lat_share.py tests/test_gpu_vtile.py tests/test_gpu_stream_parity.py -q -rA --timeout 300 --timeout-method thread" \
      "pq2800:120:TXNS=2800 FDGPU_LIB=build/ab/pp.so python tools/prep_probe.py > $d/pq2800.json" \
      "po2800:120:QUAD_SHA=-1 TXNS=2800 FDGPU_LIB=build/ab/pp.so python tools/prep_probe.py > $d/po2800.json" \
      "pq1000:120:TXNS=1000 FDGPU_LIB=build/ab/pp.so python tools/prep_probe.py > $d/pq1000.json" \
      "po1000:120:QUAD_SHA=-1 TXNS=1000 FDGPU_LIB=build/ab/pp.so python tools/prep_probe.py > $d/po1000.json" \
      "pq8192:120:TXNS=8192 FDGPU_LIB=build/ab/pp.so python tools/prep_probe.py > $d/pq8192.json" \
      "po8192:120:QUAD_SHA=-1 TXNS=8192 FDGPU_LIB=build/ab/pp.so python tools/prep_probe.py > $d/po8192.json" \
      "trace2800:180:FDGPU_LIB=firedancer_amd/libfdgpu_ed25519.so TXNS=2800 rocprofv3 --kernel-trace --stats -f csv -d $d/trace -o run -- python3 tools/prep_probe.py" &&
    run_arms r05_qs "$Q --stream-only-paced --stream-rates 5e6,7.5e6,10e6,12.5e6 --stream-paced-seconds 3" \
      "q1=" "o1=--stream-quad-sha -1" "q2=" "o2=--stream-quad-sha -1"
    ;;
  pf)
    # paced legs: the tile's prefetch distance (own frags ahead: mcache line and record header), 1 (default) vs 4 / 8
    run_arms r05_pf "$Q --stream-only-paced --stream-rates 5e6,7.5e6,10e6,12.5e6 --stream-paced-seconds 3" \
      "p1a=" "p8a=--stream-pf-dist 8" "p4a=--stream-pf-dist 4" "p1b=" "p8b=--stream-pf-dist 8" "p4b=--stream-pf-dist 4"
    ;;
  lq2)
    # gather delays split at the runtime call (issue -> start on the GPU vs the launch thread's queue): default
    # paced arms and arms without the launch thread
    run_arms r05_lq2 "$Q --stream-only-paced --stream-rates 5e6,7.5e6,10e6,12.5e6 --stream-paced-seconds 3" \
      "q1=" "n1=--stream-lat-launcher 0" "q2=" "n2=--stream-lat-launcher 0" "q3=" "n3=--stream-lat-launcher 0"
    ;;
  lq)
    # the launch thread's longest runtime call per paced leg; paced arms: default, latency path up to the batch
    # limit (8192), three engine contexts per tile (each walk within 1/3 of the CUs), both
    run_arms r05_lq "$Q --stream-only-paced --stream-rates 5e6,7.5e6,10e6,12.5e6 --stream-paced-seconds 3" \
      "q1=" "m1=--stream-lat-small-max 8192" "c1=--stream-lat-ctx 3" "cm1=--stream-lat-ctx 3 --stream-lat-small-max 8192" \
      "q2=" "m2=--stream-lat-small-max 8192" "c2=--stream-lat-ctx 3" "cm2=--stream-lat-ctx 3 --stream-lat-small-max 8192"
    ;;
  cb2)
    # more interleaved pairs of the cb arms (share 1/2 vs none), after the share's own test
    bash tools/gpu_job.sh \
      "tests:300:python -u -m pytest tests/test_gpu_lat_share.py -q -rA --timeout 300 --timeout-method thread" &&
    run_arms r05_cb2 "$Q --stream-only-paced --stream-rates 5e6,7.5e6,10e6,12.5e6 --stream-paced-seconds 3" \
      "s1d=--stream-lat-share -1" "s0d=" "s1e=--stream-lat-share -1" "s0e=" "s1f=--stream-lat-share -1" "s0f=" \
      "s1g=--stream-lat-share -1" "s0g="
    ;;
  cb)
    # the exclusive walk within each context's CU share (fdgpu_ed25519_set_lat_share, --stream-lat-share): its
    # tests, the paced tile / stream parity tests, then interleaved paced-only arms, share 1/2 (default) vs none
    bash tools/gpu_job.sh \
      "tests:900:python -u -m pytest tests/test_gpu_lat_share.py tests/test_gpu_stream_parity.py tests/test_gpu_vtile.py -k 'lat_share or paced or multictx or cu_split or vs_model' -q -rA --timeout 300 --timeout-method thread" &&
    run_arms r05_cb "$Q --stream-only-paced --stream-rates 2e6,5e6,7.5e6,10e6,12.5e6 --stream-paced-seconds 3" \
      "s0a=" "s1a=--stream-lat-share -1" "s0b=" "s1b=--stream-lat-share -1" "s0c=" "s1c=--stream-lat-share -1"
    ;;
  pp)
    d="gpurun_out/r05_pp"; mkdir -p "$d"
    bash tools/gpu_job.sh \
      "parity:900:python -u -m pytest tests/test_gpu_stream_parity.py tests/test_gpu_vtile.py -k 'paced or launch or multictx' -q -rA --timeout 300 --timeout-method thread" \
      "pp2800:120:TXNS=2800 FDGPU_LIB=build/ab/pp.so python tools/prep_probe.py > $d/pp2800.json" \
      "pp1000:120:TXNS=1000 FDGPU_LIB=build/ab/pp.so python tools/prep_probe.py > $d/pp1000.json" \
      "pp8192:120:TXNS=8192 FDGPU_LIB=build/ab/pp.so python tools/prep_probe.py > $d/pp8192.json" \
      "trace2800:180:FDGPU_LIB=firedancer_amd/libfdgpu_ed25519.so TXNS=2800 rocprofv3 --kernel-trace --stats -f csv -d $d/trace -o run -- python3 tools/prep_probe.py" &&
    run_arms r05_lc "$Q --stream-rates 5e6,7.5e6,10e6,12.5e6,15e6 --stream-paced-seconds 3 --stream-seconds 3 --stream-unrel-seconds 1" \
      "l0a=--stream-lat-launcher 0" "l1a=--stream-lat-launcher 1" "l1b=--stream-lat-launcher 1" "l0b=--stream-lat-launcher 0"
    ;;
  hc)
    # host copy threads (--stream-copy-threads): the parity tests, then max-rate arms on 2 and 3 tiles
    bash tools/gpu_job.sh \
      "parity:900:python -u -m pytest tests/test_gpu_stream_parity.py tests/test_gpu_vtile.py -k 'host or copy_threads or vs_model' -q -rA --timeout 300 --timeout-method thread" &&
    run_arms r05_hc "$Q --stream-rates 10e6 --stream-paced-seconds 3 --stream-seconds 4 --stream-unrel-seconds 2" \
      "b0a=" "h1a=--stream-copy-threads 1" "h2a=--stream-copy-threads 2" "t3h2a=--stream-tiles 3 --stream-copy-threads 2" \
      "t3h1a=--stream-tiles 3 --stream-copy-threads 1" "t4h1a=--stream-tiles 4 --stream-copy-threads 1" \
      "h2b=--stream-copy-threads 2" "b0b="
    ;;
  hc2)
    # copy threads with streaming stores, grouped publishes and cached counters; max-rate batches held to the
    # throughput path (--stream-tput-min-batch 40960)
    M="--stream-tput-min-batch 40960"
    bash tools/gpu_job.sh \
      "parity:900:python -u -m pytest tests/test_gpu_stream_parity.py tests/test_gpu_vtile.py -k 'host or copy_threads' -q -rA --timeout 300 --timeout-method thread" &&
    run_arms r05_hc2 "$Q --stream-rates 10e6 --stream-paced-seconds 3 --stream-seconds 4 --stream-unrel-seconds 2" \
      "b0a=" "m0a=$M" "h2ma=--stream-copy-threads 2 $M" "t3h2ma=--stream-tiles 3 --stream-copy-threads 2 $M" \
      "t3h1ma=--stream-tiles 3 --stream-copy-threads 1 $M" "t4h1ma=--stream-tiles 4 --stream-copy-threads 1 $M" \
      "h3ma=--stream-copy-threads 3 $M" "h2mb=--stream-copy-threads 2 $M" "t3h2mb=--stream-tiles 3 --stream-copy-threads 2 $M" "b0b="
    ;;
  hc3)
    # copy threads with plain copies and a whole-record prefetch; max-rate batches above 8K signatures on the
    # throughput path (--stream-tput-small-max 8192)
    S="--stream-tput-small-max 8192"
    bash tools/gpu_job.sh \
      "parity:900:python -u -m pytest tests/test_gpu_stream_parity.py tests/test_gpu_vtile.py -k 'host or copy_threads' -q -rA --timeout 300 --timeout-method thread" \
      "pp2:120:mkdir -p gpurun_out/r05_pp && PROBE_NOCHECK=1 TXNS=2800 FDGPU_LIB=build/ab/pp2.so python tools/prep_probe.py > gpurun_out/r05_pp/pp2800_sha_only.json" \
      "pp3:120:PROBE_NOCHECK=1 TXNS=2800 FDGPU_LIB=build/ab/pp3.so python tools/prep_probe.py > gpurun_out/r05_pp/pp2800_to_k.json" &&
    run_arms r05_hc3 "$Q --stream-rates 10e6 --stream-paced-seconds 3 --stream-seconds 4 --stream-unrel-seconds 2" \
      "b0a=" "s0a=$S" "h2sa=--stream-copy-threads 2 $S" "t3h2sa=--stream-tiles 3 --stream-copy-threads 2 $S" \
      "t3h3sa=--stream-tiles 3 --stream-copy-threads 3 $S" "t4h2sa=--stream-tiles 4 --stream-copy-threads 2 $S" \
      "t3h2sb=--stream-tiles 3 --stream-copy-threads 2 $S" "h2sb=--stream-copy-threads 2 $S" "b0b="
    ;;
  pp45)
    # the hash role split further: up to the lattice reduction (pp4), up to s' without the digits (pp5)
    mkdir -p gpurun_out/r05_pp
    bash tools/gpu_job.sh \
      "pp4:120:PROBE_NOCHECK=1 TXNS=2800 FDGPU_LIB=build/ab/pp4.so python tools/prep_probe.py > gpurun_out/r05_pp/pp2800_to_lattice.json" \
      "pp5:120:PROBE_NOCHECK=1 TXNS=2800 FDGPU_LIB=build/ab/pp5.so python tools/prep_probe.py > gpurun_out/r05_pp/pp2800_to_sprime.json"
    ;;
  hk)
    # the paced tile's housekeeping interval (launch decision, early copies, verdict poll): 10 (default) / 5 /
    # 2.5 us, and 2.5 us with the launch thread (its launches then cost the tile a queue push)
    run_arms r05_hk "$Q --stream-rates 7.5e6,10e6,12.5e6 --stream-paced-seconds 3 --stream-seconds 3 --stream-unrel-seconds 1" \
      "k10a=" "k2a=--stream-lat-hk-us 2.5" "k5a=--stream-lat-hk-us 5" "k2la=--stream-lat-hk-us 2.5 --stream-lat-launcher 1" \
      "k2lb=--stream-lat-hk-us 2.5 --stream-lat-launcher 1" "k5b=--stream-lat-hk-us 5" "k2b=--stream-lat-hk-us 2.5" "k10b="
    ;;
  sl)
    # the latency path's slow list run at the end of the 8/4/2-lane walks (one kernel less on the chain): the
    # engine-path parity tests, then interleaved A/B against the previous build (build/ab/old: engine + tile)
    # -- device batch latency (tools/latency_probe.py) and paced legs
    d=gpurun_out/r05_sl; mkdir -p $d
    O="FDGPU_LIB=build/ab/old/libfdgpu_ed25519.so FDGPU_VTILE_LIB=build/ab/old/libfdgpu_vtile.so"
    P="$Q --stream-only-paced --stream-rates 5e6,7.5e6,10e6,12.5e6 --stream-paced-seconds 3"
    bash tools/gpu_job.sh \
      "tests:900:python -u -m pytest tests/test_gpu_edges.py tests/test_gpu_parity.py tests/test_gpu_hs_top.py tests/test_gpu_lat_share.py tests/test_gpu_vtile.py tests/test_gpu_stream_parity.py -q -rA --timeout 300 --timeout-method thread" \
      "lpn1:200:python tools/latency_probe.py 1024 2800 8192 > $d/lpn1.out" \
      "lpo1:200:env $O python tools/latency_probe.py 1024 2800 8192 > $d/lpo1.out" \
      "lpn2:200:python tools/latency_probe.py 1024 2800 8192 > $d/lpn2.out" \
      "lpo2:200:env $O python tools/latency_probe.py 1024 2800 8192 > $d/lpo2.out" \
      "n1:240:python3 bench.py $P --detail-out $d/n1.json > $d/n1.out" \
      "o1:240:env $O python3 bench.py $P --detail-out $d/o1.json > $d/o1.out" \
      "n2:240:python3 bench.py $P --detail-out $d/n2.json > $d/n2.out" \
      "o2:240:env $O python3 bench.py $P --detail-out $d/o2.json > $d/o2.out"
    ;;
  lw)
    # the throughput walk's last partial round: a 1M batch is 16 waves per SIMD, which at the register limit's
    # 3 waves per SIMD run as 5 rounds and a lone wave.  Arms: default; 2 workgroups per CU by an LDS
    # reservation (build/ab/l2.so, FD_DSMH_LDS=57344: 8 full rounds); the unfolded walk (2 waves per SIMD by
    # its registers, FDGPU_NOFOLD_MAX)
    d=gpurun_out/r05_lw; mkdir -p $d
    H="python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --latency-batch 0 --stream-frags 0 --no-extra-configs"
    bash tools/gpu_job.sh \
      "b1:200:$H --detail-out $d/b1.json > $d/b1.out" \
      "l1:200:FDGPU_LIB=build/ab/l2.so $H --detail-out $d/l1.json > $d/l1.out" \
      "n1:200:FDGPU_NOFOLD_MAX=2000000 $H --detail-out $d/n1.json > $d/n1.out" \
      "b2:200:$H --detail-out $d/b2.json > $d/b2.out" \
      "l2:200:FDGPU_LIB=build/ab/l2.so $H --detail-out $d/l2.json > $d/l2.out" \
      "n2:200:FDGPU_NOFOLD_MAX=2000000 $H --detail-out $d/n2.json > $d/n2.out" \
      "ktl:200:FDGPU_LIB=build/ab/l2.so rocprofv3 --kernel-trace --stats -f csv -d $d/kl -o run -- $H > $d/kl.out"
    ;;
  fin)
    # round-end evidence, second half (the GPU suite and smoke ran in a call of their own, profiles/r05/final5):
    # tools/gpu_final.sh's bench, rocprof stats and PMC passes (TAG=final7: the GPU suite and smoke first)
    tag=${TAG:-final5}; d="gpurun_out/prof_$tag"; mkdir -p $d
    if [ -n "$TAG" ]; then
      bash tools/gpu_job.sh \
        "tests:900:python -u -m pytest tests -m gpu -q -rA --timeout 300 --timeout-method thread" \
        "smoke:200:python -c 'import __graft_entry__ as g; g.smoke(); print(\"smoke ok\")'" || exit $?
    fi
    B="python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --latency-batch 0 --stream-frags 0 --no-extra-configs"
    P="timeout -s KILL 120 rocprofv3 --kernel-include-regex fd_ -f csv"
    bash tools/gpu_job.sh \
      "bench:480:python bench.py --steps 20 --warmup 5 --detail-out $d/bench_detail.json > gpurun_out/bench_$tag.json" \
      "stats:180:rocprofv3 --kernel-trace --stats -f csv -d $d/stats -o run -- $B > $d/bench_under_rocprof.json" \
      "pmc_fetch:150:$P --pmc FETCH_SIZE -d $d/fetch -o run -- $B" \
      "pmc_write:150:$P --pmc WRITE_SIZE -d $d/write -o run -- $B" \
      "pmc_sq:150:$P --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAVES GRBM_GUI_ACTIVE -d $d/sq -o run -- $B"
    ;;
  *) sed -n '2,8p' "$0"; exit 2 ;;
esac
