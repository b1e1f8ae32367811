#!/bin/bash
# r04: fp32 GEMM autotune breadth at config 3: the default candidate count against 32 / 64
# hipBLASLt heuristics (DCN_GEMM_CANDIDATES), two runs each on one box.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${1:-gc}
run() {  # name env...
  local name=$1; shift
  env "$@" timeout -k 10 150 python bench.py --config 3 --steps 20 --warmup 5 --no-cpu-baseline --no-strong --no-host-path --no-config4 --alt-math 0 > gpurun_out/${T}_$name.json 2> gpurun_out/${T}_$name.err || { tail -5 gpurun_out/${T}_$name.err; exit 1; }
  python -c "import json,sys; d=json.loads(open('gpurun_out/${T}_$name.json').read().splitlines()[-1]); print('$name', d['ms_per_step'], {k: d['kernel_ms'].get(k) for k in ('gemm_fwd','gemm_dw','gemm_dcol')})"
}
for rep in 1 2; do
  run c8_$rep DCN_DUMMY=0
  run c32_$rep DCN_GEMM_CANDIDATES=32
  run c64_$rep DCN_GEMM_CANDIDATES=64
done
echo gc done
