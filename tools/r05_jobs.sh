#!/bin/bash
# Round-5 GPU jobs: tools/r05_jobs.sh <job>   (each step under its own time limit via tools/gpu_job.sh)
#   pp     : prep role lengths of latency-path batches (FD_PREP_PROBE variant, tools/prep_probe.py) + the
#            chain's kernel trace at 2,800 txns, and the paced two-context stream parity tests
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
job="$1"; shift
d="gpurun_out/r05_$job"; mkdir -p "$d"
case "$job" in
  pp)
    bash tools/gpu_job.sh \
      "parity:900:python -u -m pytest tests/test_gpu_stream_parity.py -k paced -q --timeout 300 --timeout-method thread" \
      "pp2800:120:TXNS=2800 python tools/prep_probe.py > $d/pp2800.json" \
      "pp1000:120:TXNS=1000 python tools/prep_probe.py > $d/pp1000.json" \
      "pp8192:120:TXNS=8192 python tools/prep_probe.py > $d/pp8192.json" \
      "trace2800:180:FDGPU_LIB=firedancer_amd/libfdgpu_ed25519.so TXNS=2800 rocprofv3 --kernel-trace --stats -f csv -d $d/trace -o run -- python3 tools/prep_probe.py"
    ;;
  *) echo "unknown job $job"; exit 2 ;;
esac
