#!/bin/bash
# r04: K5 batched ∂offset tree (4 waves/SIMD), fp32 offset conv (row-broadcast VALU weights in the
# forward, 32x32x2 ∂W_off kernel), warp-specialised bf16 kernels reverted. Parity first, then
# A/B against tools/alt/alt0 (the r03 K5 and offset conv; its fused bf16 kernels pinned to the
# r03 ones) and tools/alt/nopp (this build without the K5 register-set alternation), a bitwise dump comparison, and the whole GPU suite. Stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${1:-oc}
ALT0="DCN_LIB=tools/alt/alt0/libdcn.so DCN_FWD_WS=0 DCN_DW_WS=0"
echo "== parity" && \
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_bf16.py tests/test_gpu_fused_bf16.py -x -q --timeout 120 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1 || { tail -40 gpurun_out/${T}_pytest.log; exit 1; }
tail -2 gpurun_out/${T}_pytest.log
run() {  # name env...
  local name=$1; shift
  env "$@" timeout -k 10 120 python bench.py --config ${CFG:-3} --steps 20 --warmup 5 --no-cpu-baseline --no-strong --no-host-path --no-config4 > gpurun_out/${T}_$name.json 2> gpurun_out/${T}_$name.err || { tail -5 gpurun_out/${T}_$name.err; exit 1; }
  python -c "import json,sys; d=json.loads(open('gpurun_out/${T}_$name.json').read().splitlines()[-1]); print('$name', d['ms_per_step'], {k: d['kernel_ms'].get(k) for k in ('offset_fwd','offset_bwd','col2im','gemm_fwd','gemm_dw')})"
}
for rep in 1 2; do
  for c in 3 4; do
    CFG=$c run r03_c${c}_$rep $ALT0
    CFG=$c run new_c${c}_$rep DCN_DUMMY=0
    CFG=$c run nopp_c${c}_$rep DCN_LIB=tools/alt/nopp/libdcn.so
  done
done
echo "== bitwise dumps (alt0 vs this build)" && \
env $ALT0 timeout -k 10 300 python tools/ab_bitwise.py dump /tmp/ab_a.npz > gpurun_out/${T}_ab.log 2>&1 && \
timeout -k 10 300 python tools/ab_bitwise.py dump /tmp/ab_b.npz >> gpurun_out/${T}_ab.log 2>&1 && \
timeout -k 10 120 python tools/ab_bitwise.py cmp /tmp/ab_a.npz /tmp/ab_b.npz >> gpurun_out/${T}_ab.log 2>&1; tail -30 gpurun_out/${T}_ab.log
echo "== pytest -m gpu" && \
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${T}_pytest_all.log 2>&1 || { tail -40 gpurun_out/${T}_pytest_all.log; exit 1; }
tail -3 gpurun_out/${T}_pytest_all.log
