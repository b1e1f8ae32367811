#!/bin/bash
# r04: ∂W grouping A/B at config 4 (16 groups = this build, 32 = tools/alt/g32), then SQ counters
# at config 3 (K5, offset conv) and HBM traffic at config 4 for both groupings. Stops at the
# first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${1:-pm}
run() {  # name env...
  local name=$1; shift
  env "$@" timeout -k 10 120 python bench.py --config 4 --steps 20 --warmup 5 --no-cpu-baseline --no-strong --no-host-path --no-config4 > gpurun_out/${T}_$name.json 2> gpurun_out/${T}_$name.err || { tail -5 gpurun_out/${T}_$name.err; exit 1; }
  python -c "import json,sys; d=json.loads(open('gpurun_out/${T}_$name.json').read().splitlines()[-1]); print('$name', d['ms_per_step'], {k: d['kernel_ms'].get(k) for k in ('gemm_fwd','gemm_dw','gemm_dcol','col2im','offset_bwd')})"
}
echo "== bitwise dumps, GEMM choice pinned (alt0 = r03 K5 / offset conv vs this build)" && \
PIN="DCN_GEMM_BACKEND=hipblaslt DCN_GEMM_CANDIDATES=1" && \
env $PIN DCN_LIB=tools/alt/alt0/libdcn.so DCN_FWD_WS=0 DCN_DW_WS=0 timeout -k 10 300 python tools/ab_bitwise.py dump /tmp/ab_a.npz > gpurun_out/${T}_ab.log 2>&1 && \
env $PIN timeout -k 10 300 python tools/ab_bitwise.py dump /tmp/ab_b.npz >> gpurun_out/${T}_ab.log 2>&1 && \
timeout -k 10 120 python tools/ab_bitwise.py cmp /tmp/ab_a.npz /tmp/ab_b.npz >> gpurun_out/${T}_ab.log 2>&1; grep -v "bitwise equal" gpurun_out/${T}_ab.log | tail -12
rm -f /tmp/ab_a.npz /tmp/ab_b.npz
for rep in 1 2; do
  run g16_$rep DCN_DUMMY=0
  run g32_$rep DCN_LIB=tools/alt/g32/libdcn.so
done
echo "== SQ counters, config 3" && bash tools/pmc_sq.sh ${T}c3 && \
echo "== HBM traffic, config 4 (16 groups, 32 groups)" && BENCH_ARGS="--config 4" bash tools/pmc_pass.sh ${T}c4g16 && \
DCN_LIB=tools/alt/g32/libdcn.so BENCH_ARGS="--config 4" bash tools/pmc_pass.sh ${T}c4g32 && echo pmc all done
