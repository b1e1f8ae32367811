#!/bin/bash
# r04: the side stream (bins, ∂W partial fold, channel sums) at the lowest stream priority
# (tools/alt/auxlo) against this build (default priority), configs 3 and 4, after parity.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${1:-aux}
DCN_LIB=tools/alt/auxlo/libdcn.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_bf16.py -x -q --timeout 120 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1 || { tail -20 gpurun_out/${T}_pytest.log; exit 1; }
echo "auxlo parity: $(tail -1 gpurun_out/${T}_pytest.log)"
run() {  # name env...
  local name=$1; shift
  env "$@" timeout -k 10 120 python bench.py --config ${CFG:-4} --steps 20 --warmup 5 --no-cpu-baseline --no-strong --no-host-path --no-config4 --alt-math 0 > gpurun_out/${T}_$name.json 2> gpurun_out/${T}_$name.err || { tail -5 gpurun_out/${T}_$name.err; exit 1; }
  python -c "import json,sys; d=json.loads(open('gpurun_out/${T}_$name.json').read().splitlines()[-1]); print('$name', d['ms_per_step'], {k: d['kernel_ms'].get(k) for k in ('gemm_dw','gemm_dcol','col2im','bwd_bias')})"
}
for rep in 1 2; do
  for c in 3 4; do
    CFG=$c run cur_c${c}_$rep DCN_DUMMY=0
    CFG=$c run auxlo_c${c}_$rep DCN_LIB=tools/alt/auxlo/libdcn.so
  done
done
echo aux done
