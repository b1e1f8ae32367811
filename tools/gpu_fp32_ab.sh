#!/bin/bash
# fp32 backward change check: fp32 parity suites, then three config-3 benches.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_sweep.py tests/test_gpu_ednet.py tests/test_gpu_fused.py -x -q --timeout 120 --timeout-method thread > gpurun_out/fp32_t.log 2>&1 || { tail -30 gpurun_out/fp32_t.log; exit 1; }
tail -n1 gpurun_out/fp32_t.log
for i in 1 2 3; do
  timeout -k 10 120 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --alt-math 0 > gpurun_out/fp32_b$i.json || exit 1
  python -c "import json; d=json.load(open('gpurun_out/fp32_b$i.json')); k=d['kernel_ms']; print(d['ms_per_step'], k['bwd_bias'], k['gemm_dw'])"
done
