#!/bin/bash
# bf16 parity tests and a config-4 bench (after a bf16-path change).
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_bf16.py -x -q --timeout 120 --timeout-method thread > gpurun_out/bf16_t.log 2>&1 || { tail -30 gpurun_out/bf16_t.log; exit 1; }
tail -n1 gpurun_out/bf16_t.log
for i in 1 2; do
  timeout -k 10 120 python bench.py --config 4 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bf16_b$i.json || exit 1
  python -c "import json; d=json.load(open('gpurun_out/bf16_b$i.json')); print(d['ms_per_step'], d['kernel_ms'])"
done
