#!/bin/bash
# ∂W GEMM grouping A/B (DCN_EXP slot 9 = groups, 0 = one GEMM per image): parity tests with
# the grouped path forced, then config 3 and config 4 benches per grouping.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
E="0,0,0,0,0,0,0,0,0"  # slot 9 follows: n>0 groups, -1 per image, 0 default
DCN_EXP="$E,1" timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_bf16.py -x -q --timeout 120 --timeout-method thread > gpurun_out/dw_t.log 2>&1 || { tail -20 gpurun_out/dw_t.log; exit 1; }
for n in 0 2 4 8 16; do
  DCN_EXP="$E,$n" timeout -k 10 120 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --alt-math 0 > gpurun_out/dw3_$n.json || exit 1
  DCN_EXP="$E,$n" timeout -k 10 120 python bench.py --config 4 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/dw4_$n.json || exit 1
done
echo dw done
