#!/bin/bash
# hipBLASLt candidate-count A/B for the config-4 bf16 GEMMs (DCN_GEMM_CANDIDATES).
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
set -o pipefail
for c in 8 64; do
  DCN_GEMM_CANDIDATES=$c timeout -k 10 200 python bench.py --config 4 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/cand4_$c.json || exit 1
  python -c "import json; d=json.load(open('gpurun_out/cand4_$c.json')); k=d['kernel_ms']; print($c, d['ms_per_step'], k['gemm_fwd'], k['gemm_dw'], k['gemm_dcol'])"
done
