#!/bin/bash
# r04: diagnosis of the warp-specialised bf16 kernels (temporary DCN_WS_DBG knob: 1 producers skip
# the gather, 2 consumers skip the MFMAs, 4 scalar blend, 8 16-B column stores) at config 4,
# after their parity tests. Stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${1:-ws2}
echo "== fused bf16 parity" && \
timeout -k 10 240 python -u -m pytest tests/test_gpu_fused_bf16.py -x -q --timeout 100 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1 || { tail -30 gpurun_out/${T}_pytest.log; exit 1; }
tail -2 gpurun_out/${T}_pytest.log
run() {  # name env... -- bench args
  local name=$1; shift
  env "$@" timeout -k 10 120 python bench.py --config ${CFG:-4} --steps 20 --warmup 5 --no-cpu-baseline --no-strong --no-host-path $BARGS > gpurun_out/${T}_$name.json 2> gpurun_out/${T}_$name.err || { tail -5 gpurun_out/${T}_$name.err; exit 1; }
  python -c "import json,sys; d=json.loads(open('gpurun_out/${T}_$name.json').read().splitlines()[-1]); print('$name', d['ms_per_step'], {k: d['kernel_ms'].get(k) for k in ('gemm_fwd','gemm_dw','col2im','im2col')})"
}
for fp in 2 3; do
  BARGS="--fwd-path $fp"
  run old_p$fp DCN_FWD_WS=0 DCN_DW_WS=0
  for v in 0 4 1 2 5; do run ws_p${fp}_d$v DCN_WS_DBG=$v; done
  run old2_p$fp DCN_FWD_WS=0 DCN_DW_WS=0
done
BARGS="--no-config4"
for rep in 1 2; do  # K5 A/B: r03 K5 (alt0), batched-butterfly K5 (alt1), product (bitwise batched tree)
  for c in 3 4; do
    CFG=$c run k5old_c${c}_$rep DCN_LIB=tools/alt/alt0/libdcn.so
    CFG=$c run k5nb_c${c}_$rep DCN_LIB=tools/alt/alt1/libdcn.so
    CFG=$c run k5new_c${c}_$rep DCN_DUMMY=0
  done
done
echo variants done
echo "== pytest -m gpu" && \
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${T}_pytest_all.log 2>&1 || { tail -30 gpurun_out/${T}_pytest_all.log; exit 1; }
tail -3 gpurun_out/${T}_pytest_all.log
echo "== launch_diag" && \
timeout -k 10 240 python -u tools/launch_diag.py --reps 200 --reps3 40 --out gpurun_out/${T}_diag.json > gpurun_out/${T}_diag.log 2>&1 || { tail -3 gpurun_out/${T}_diag.log | cut -c1-800; exit 1; }
echo diag ok
echo "== bitwise A/B against the r03 K5 / offset conv (alt0)" && \
DCN_LIB=tools/alt/alt0/libdcn.so timeout -k 10 300 python tools/ab_bitwise.py dump /tmp/ab_a.npz > gpurun_out/${T}_ab.log 2>&1 && \
timeout -k 10 300 python tools/ab_bitwise.py dump /tmp/ab_b.npz >> gpurun_out/${T}_ab.log 2>&1 && \
python tools/ab_bitwise.py cmp /tmp/ab_a.npz /tmp/ab_b.npz >> gpurun_out/${T}_ab.log 2>&1; tail -40 gpurun_out/${T}_ab.log
