#!/bin/bash
# Round-6 GPU jobs: tools/r06_jobs.sh <job>   (each step under its own time limit via tools/gpu_job.sh)
#   first : the restored tree: default bench (line + detail) and the stream / tile parity tests
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
job="$1"; shift
T="python -u -m pytest -q -rA --timeout 300 --timeout-method thread"

case "$job" in
  first)
    d=gpurun_out/r06_first; mkdir -p $d
    bash tools/gpu_job.sh \
      "bench:400:python bench.py --detail-out $d/bench_detail.json > $d/bench_line.json" \
      "tests:600:$T tests/test_gpu_stream_parity.py tests/test_gpu_vtile.py tests/test_gpu_stem.py"
    ;;
  svc)
    # the verify service: its GPU tests (served tile processes against the reference tile, fault path, numa lookup,
    # the launch-thread failure), then paced curves with T = 1, 2, 3 tile processes per GPU next to the default legs
    d=gpurun_out/r06_svc; mkdir -p $d
    bash tools/gpu_job.sh \
      "tests:700:$T tests/test_gpu_vsvc.py" \
      "bench:600:python bench.py --steps 2 --warmup 1 --txns 262144 --no-cpu-baseline --no-extra-configs --latency-batch 0 --stream-svc-tiles 1,2,3 --detail-out $d/detail.json > $d/line.json"
    ;;
  svc2)
    d=gpurun_out/r06_svc2; mkdir -p $d
    bash tools/gpu_job.sh \
      "bench:600:python bench.py --steps 2 --warmup 1 --txns 262144 --no-cpu-baseline --no-extra-configs --latency-batch 0 --stream-svc-tiles 1,2,3 --detail-out $d/detail.json > $d/line.json" \
      "tests:600:$T tests/test_gpu_stream_parity.py -k 'reliable and not launch and not host'"
    ;;
  cmp)
    # paced curves at equal device load: one tile process with its engine contexts (A), T = 1, 2, 3 served tile
    # processes (A), and two tile processes each with a GPU context of its own (the N = 2 rehearsal on one
    # device: per-rank rates half the device's), then A again
    d=gpurun_out/r06_cmp; mkdir -p $d
    A="python bench.py --steps 2 --warmup 1 --txns 262144 --no-cpu-baseline --no-extra-configs --latency-batch 0 --stream-only-paced --stream-svc-tiles 1,2,3"
    bash tools/gpu_job.sh \
      "a1:400:$A --detail-out $d/a1.json > $d/a1.line" \
      "own2:400:bash tools/rehearse_n2.sh --stream-only-paced --stream-rates 1e6,2.5e6,3.75e6,5e6,7.5e6 --no-cpu-baseline --detail-out $d/own2.json > $d/own2.line" \
      "a2:400:$A --detail-out $d/a2.json > $d/a2.line"
    ;;
  m1)
    # the sandbox measurements, then the paced comparison (job cmp)
    bash tools/gpu_sandbox.sh gpurun_out/r06_sandbox && bash tools/r06_jobs.sh cmp
    ;;
  place)
    # the link's NUMA placement: producer + its mcache and dcache part on the GPU's node vs on the other node
    # (the cross-socket arm), interleaved: max rate, intake ns/frag, gather GB/s, paced p99 at 10M
    d=gpurun_out/r06_place; mkdir -p $d
    P="python bench.py --steps 2 --warmup 1 --txns 262144 --no-cpu-baseline --no-extra-configs --latency-batch 0 --stream-rates 10e6 --stream-seconds 5 --stream-unrel-seconds 1"
    bash tools/gpu_job.sh \
      "g1:300:$P --stream-place gpu --detail-out $d/g1.json > $d/g1.line" \
      "o1:300:$P --stream-place opposite --detail-out $d/o1.json > $d/o1.line" \
      "g2:300:$P --stream-place gpu --detail-out $d/g2.json > $d/g2.line" \
      "o2:300:$P --stream-place opposite --detail-out $d/o2.json > $d/o2.line"
    ;;
  n2svc)
    # the N = 2 flow with served legs, both ranks on one GPU (each rank's stream child is the verify service of
    # its GPU and starts its own tile processes; the link is shared through /dev/shm): correctness of the G > 1
    # served path (two services on one device contend, as two GPUs' would not)
    d=gpurun_out/r06_n2svc; mkdir -p $d
    bash tools/gpu_job.sh \
      "n2:500:bash tools/rehearse_n2.sh --stream-only-paced --stream-rates 1e6,2.5e6 --stream-svc-tiles 1,2 --no-cpu-baseline --detail-out $d/detail.json > $d/line.json"
    ;;
  dflt)
    # the default bench (served legs included) timed end to end, then the served tests
    d=gpurun_out/r06_dflt; mkdir -p $d
    bash tools/gpu_job.sh \
      "bench:600:python bench.py --detail-out $d/detail.json > $d/line.json" \
      "tests:600:$T tests/test_gpu_vsvc.py"
    ;;
  hi)
    # served tiles above the knee: 10M, 12.5M, 15M per GPU, T = 2, 3 beside one process (twice, interleaved)
    d=gpurun_out/r06_hi; mkdir -p $d
    A="python bench.py --steps 2 --warmup 1 --txns 262144 --no-cpu-baseline --no-extra-configs --latency-batch 0 --stream-only-paced --stream-rates 10e6,12.5e6,15e6 --stream-svc-tiles 2,3"
    bash tools/gpu_job.sh \
      "h1:400:$A --detail-out $d/h1.json > $d/h1.line" \
      "h2:400:$A --detail-out $d/h2.json > $d/h2.line"
    ;;
  smax)
    # served max rate (reliable link, credit-based) with T = 2, 3, 4 tile processes beside the one-process legs
    d=gpurun_out/r06_smax; mkdir -p $d
    bash tools/gpu_job.sh \
      "s1:500:python bench.py --steps 2 --warmup 1 --txns 262144 --no-cpu-baseline --no-extra-configs --latency-batch 0 --stream-rates 10e6,12.5e6 --stream-svc-tiles 2,3,4 --stream-svc-max 1 --detail-out $d/s1.json > $d/s1.line"
    ;;
  smax2)
    # served max rate with the one-process max leg's engine contexts in the service (2), T = 2, 3, 4
    d=gpurun_out/r06_smax2; mkdir -p $d
    bash tools/gpu_job.sh \
      "s2:500:python bench.py --steps 2 --warmup 1 --txns 262144 --no-cpu-baseline --no-extra-configs --latency-batch 0 --stream-rates 10e6,12.5e6 --stream-svc-tiles 2,3,4 --stream-svc-max 1 --detail-out $d/s2.json > $d/s2.line"
    ;;
  sprof)
    # where a served tile's time goes at the max rate: the rdtsc section profile, T = 2 and 4, one process beside
    d=gpurun_out/r06_sprof; mkdir -p $d
    bash tools/gpu_job.sh \
      "p1:500:python bench.py --steps 2 --warmup 1 --txns 262144 --no-cpu-baseline --no-extra-configs --latency-batch 0 --stream-rates 10e6 --stream-svc-tiles 2,4 --stream-svc-max 1 --stream-prof --detail-out $d/p1.json > $d/p1.line"
    ;;
  db)
    # default runs of the final build, back to back
    d=gpurun_out/${FDJOB_DIR:-r06_db}; mkdir -p $d
    bash tools/gpu_job.sh \
      "d1:400:python bench.py --detail-out $d/d1.json > $d/d1.line" \
      "d2:400:python bench.py --detail-out $d/d2.json > $d/d2.line" \
      "d3:400:python bench.py --detail-out $d/d3.json > $d/d3.line"
    ;;
  soak)
    # 30-s paced legs at 10M and 12.5M per GPU: one tile process, and 2 served tile processes
    d=gpurun_out/r06_soak; mkdir -p $d
    bash tools/gpu_job.sh \
      "k1:600:python bench.py --steps 2 --warmup 1 --txns 262144 --no-cpu-baseline --no-extra-configs --latency-batch 0 --stream-only-paced --stream-rates 10e6,12.5e6 --stream-paced-seconds 30 --stream-svc-tiles 2 --detail-out $d/k1.json > $d/k1.line"
    ;;
  pages)
    # 4 KiB vs 2 MiB pages under the one-process link (--stream-no-huge), 30-s paced legs at 10M, interleaved
    d=gpurun_out/r06_pages; mkdir -p $d
    P="python bench.py --steps 2 --warmup 1 --txns 262144 --no-cpu-baseline --no-extra-configs --latency-batch 0 --stream-only-paced --stream-rates 10e6 --stream-paced-seconds 30 --stream-svc-tiles ''"
    bash tools/gpu_job.sh \
      "h1:300:$P --detail-out $d/h1.json > $d/h1.line" \
      "s1:300:$P --stream-no-huge --detail-out $d/s1.json > $d/s1.line" \
      "h2:300:$P --detail-out $d/h2.json > $d/h2.line" \
      "s2:300:$P --stream-no-huge --detail-out $d/s2.json > $d/s2.line"
    ;;
  n4svc)
    # the N = 4 flow with the default served legs (T = 2), all four ranks on one GPU: the wiring of 4 services and
    # 8 tile processes over shared links (four services on one device contend, as four GPUs' would not)
    d=gpurun_out/r06_n4svc; mkdir -p $d
    bash tools/gpu_job.sh \
      "n4:600:bash tools/rehearse_n4.sh --stream-only-paced --stream-rates 5e5,1e6 --stream-paced-seconds 2 --detail-out $d/detail.json > $d/line.json"
    ;;
  ctx3)
    # served legs above the knee with three engine contexts in the service (and the one-process tile) against the
    # default two, interleaved: does a third staggered context move the served knee past 12.5M?
    d=gpurun_out/r06_ctx3; mkdir -p $d
    A="python bench.py --steps 2 --warmup 1 --txns 262144 --no-cpu-baseline --no-extra-configs --latency-batch 0 --stream-only-paced --stream-rates 10e6,12.5e6,15e6 --stream-svc-tiles 2,3"
    bash tools/gpu_job.sh \
      "c2a:400:$A --stream-lat-ctx 2 --detail-out $d/c2a.json > $d/c2a.line" \
      "c3a:400:$A --stream-lat-ctx 3 --detail-out $d/c3a.json > $d/c3a.line" \
      "c2b:400:$A --stream-lat-ctx 2 --detail-out $d/c2b.json > $d/c2b.line" \
      "c3b:400:$A --stream-lat-ctx 3 --detail-out $d/c3b.json > $d/c3b.line"
    ;;
  hard)
    # the service serving from its own copy of the layout: its GPU tests, then the driver's own N = 2 command
    # (default flags) with both ranks on one GPU
    d=gpurun_out/r06_hard; mkdir -p $d
    bash tools/gpu_job.sh \
      "tests:600:$T tests/test_gpu_vsvc.py > $d/tests_vsvc.log 2>&1" \
      "n2:600:FDGPU_BENCH_ONE_DEVICE=1 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29535 bench.py --gpus 2 --steps 20 --warmup 5 --detail-out $d/n2_detail.json > $d/n2_line.json"
    ;;
  ftests)
    # round-end evidence, part 1: the whole GPU suite and the smoke
    d=gpurun_out/${FDJOB_DIR:-r06_final}; mkdir -p $d
    bash tools/gpu_job.sh \
      "tests:1100:$T tests -m gpu > $d/gpu_tests.log 2>&1" \
      "smoke:300:python -c 'import __graft_entry__ as g; g.smoke(); print(\"smoke ok\")' > $d/smoke.log 2>&1"
    ;;
  fbench)
    # round-end evidence, part 2: the default bench, rocprof kernel stats of the headline bench, PMC passes
    d=gpurun_out/${FDJOB_DIR:-r06_final}; mkdir -p $d
    B="python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --latency-batch 0 --stream-frags 0 --no-extra-configs"
    P="timeout -s KILL 120 rocprofv3 --kernel-include-regex fd_ -f csv"
    bash tools/gpu_job.sh \
      "bench:480:python bench.py --steps 20 --warmup 5 --detail-out $d/bench_detail.json > $d/bench_line.json" \
      "stats:240:rocprofv3 --kernel-trace --stats -f csv -d $d/stats -o run -- $B > $d/bench_under_rocprof.json" \
      "pmc_fetch:150:$P --pmc FETCH_SIZE -d $d/fetch -o run -- $B" \
      "pmc_write:150:$P --pmc WRITE_SIZE -d $d/write -o run -- $B" \
      "pmc_sq:150:$P --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAVES GRBM_GUI_ACTIVE -d $d/sq -o run -- $B"
    ;;
  svcdbg)
    bash tools/gpu_job.sh \
      "tests:300:$T -x tests/test_gpu_vsvc.py -k 'in_process or launch_thread'"
    ;;
  *) echo "unknown job $job"; exit 2 ;;
esac
