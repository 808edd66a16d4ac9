cd "${GRAFT_REPO_ROOT:-.}"
bash tools/gpu_job.sh \
  "vt:600:python -u -m pytest tests/test_gpu_vtile.py tests/test_gpu_faults.py -x -v --timeout 120 --timeout-method thread" \
  "stream:400:python bench.py --stream-child --stream-procs 1 --stream-token t1 > gpurun_out/stream1.json"
