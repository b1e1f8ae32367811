#!/bin/bash
# Split-bf16 GEMM check: its GPU tests, then bench per math mode (kernel timings).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_gemm_split.py -x -q --timeout 120 --timeout-method thread > gpurun_out/split_test.log 2>&1 || { tail -30 gpurun_out/split_test.log; exit 1; }
tail -1 gpurun_out/split_test.log
for m in ${MATHS:-0 6 9 3}; do
  timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --math $m > gpurun_out/bench_m$m.json 2>gpurun_out/bench_m$m.err || exit 1
  python -c "import json;d=json.load(open('gpurun_out/bench_m$m.json'));print($m, d['ms_per_step'], d['kernel_ms'])"
done
