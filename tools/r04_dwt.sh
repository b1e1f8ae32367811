#!/bin/bash
# r04: the bf16 ∂W GEMM transposed (P'_g(O×K) = ∂outT_g · colT_gᵀ, m = O, n = K; the partials
# summed through a transposing fixed-order fold), tools/alt/dwt, against this build (m = K,
# n = O) at config 4, after its bf16 parity tests. Stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${1:-dwt}
DCN_LIB=tools/alt/dwt/libdcn.so timeout -k 10 300 python -u -m pytest tests/test_gpu_bf16.py tests/test_gpu_fused_bf16.py -x -q --timeout 120 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1 || { tail -20 gpurun_out/${T}_pytest.log; exit 1; }
echo "dwt parity: $(tail -1 gpurun_out/${T}_pytest.log)"
run() {  # name env...
  local name=$1; shift
  env "$@" timeout -k 10 120 python bench.py --config 4 --steps 20 --warmup 5 --no-cpu-baseline --no-strong --no-host-path --no-config4 > gpurun_out/${T}_$name.json 2> gpurun_out/${T}_$name.err || { tail -5 gpurun_out/${T}_$name.err; exit 1; }
  python -c "import json,sys; d=json.loads(open('gpurun_out/${T}_$name.json').read().splitlines()[-1]); print('$name', d['ms_per_step'], {k: d['kernel_ms'].get(k) for k in ('gemm_dw','gemm_dcol','col2im')})"
}
for rep in 1 2 3; do
  run cur_$rep DCN_DUMMY=0
  run dwt_$rep DCN_LIB=tools/alt/dwt/libdcn.so
done
echo dwt done
