#!/bin/bash
# r04: bf16 offset-conv ∂x kernel with buffer-resource epilogue (121 registers, 4 workgroups per
# CU) in this build against tools/alt/pre (the same tree before it): bf16 parity, a bitwise dump
# comparison (GEMM choice pinned), config-4 A/B. Stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${1:-dg}
timeout -k 10 300 python -u -m pytest tests/test_gpu_bf16.py tests/test_gpu_fused_bf16.py tests/test_gpu_ednet.py -x -q --timeout 120 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1 || { tail -20 gpurun_out/${T}_pytest.log; exit 1; }
echo "parity: $(tail -1 gpurun_out/${T}_pytest.log)"
PIN="DCN_GEMM_BACKEND=hipblaslt DCN_GEMM_CANDIDATES=1"
env $PIN DCN_LIB=tools/alt/pre/libdcn.so timeout -k 10 300 python tools/ab_bitwise.py dump /tmp/ab_a.npz > gpurun_out/${T}_ab.log 2>&1 && \
env $PIN timeout -k 10 300 python tools/ab_bitwise.py dump /tmp/ab_b.npz >> gpurun_out/${T}_ab.log 2>&1 && \
{ timeout -k 10 120 python tools/ab_bitwise.py cmp /tmp/ab_a.npz /tmp/ab_b.npz >> gpurun_out/${T}_ab.log 2>&1; grep -v "bitwise equal" gpurun_out/${T}_ab.log | tail -4; } || exit 1
rm -f /tmp/ab_a.npz /tmp/ab_b.npz
run() {  # name env...
  local name=$1; shift
  env "$@" timeout -k 10 120 python bench.py --config 4 --steps 20 --warmup 5 --no-cpu-baseline --no-strong --no-host-path --no-config4 > gpurun_out/${T}_$name.json 2> gpurun_out/${T}_$name.err || { tail -5 gpurun_out/${T}_$name.err; exit 1; }
  python -c "import json,sys; d=json.loads(open('gpurun_out/${T}_$name.json').read().splitlines()[-1]); print('$name', d['ms_per_step'], {k: d['kernel_ms'].get(k) for k in ('offset_bwd','col2im','gemm_dw')})"
}
for rep in 1 2 3; do
  run new_$rep DCN_DUMMY=0
  run pre_$rep DCN_LIB=tools/alt/pre/libdcn.so
done
echo dg done
