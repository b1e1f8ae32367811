#!/bin/bash
# Fused-forward workgroup shapes (DCN_EXP slot 8 = 1: shape 0, else shape 1): parity tests and a config-3 bench
# of each, then the unfused schedule for reference.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for c in 0 1; do
  DCN_EXP="0,0,0,0,0,0,0,0,$c" timeout -k 10 240 python -u -m pytest tests/test_gpu_fused.py -x -q --timeout 120 --timeout-method thread > gpurun_out/fused_t$c.log 2>&1 || { tail -5 gpurun_out/fused_t$c.log; exit 1; }
  DCN_EXP="0,0,0,0,0,0,0,0,$c" timeout -k 10 120 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --alt-math 0 --fwd-path 2 > gpurun_out/fx$c.json || exit 1
done
timeout -k 10 120 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --alt-math 0 --fwd-path 1 > gpurun_out/fxu.json
