#!/bin/bash
# r04: bf16 K5 rows per batch: this build (U 4, rows widened at batch start) against
# tools/alt/k5u4g (U 4, rows widened where used, several 8-sum trees per batch), k5u6 and k5u8
# (bf16 U 6 / 8; fp32 stays U 4), with r03's K5 (tools/alt/alt0) as the reference; each alt
# first passes the parity tests. Stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${1:-k5b}
for a in k5u4g k5u6 k5u8; do
  DCN_LIB=tools/alt/$a/libdcn.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_bf16.py -x -q --timeout 120 --timeout-method thread > gpurun_out/${T}_pytest_$a.log 2>&1 || { tail -20 gpurun_out/${T}_pytest_$a.log; exit 1; }
  echo "$a parity: $(tail -1 gpurun_out/${T}_pytest_$a.log)"
done
run() {  # name env...
  local name=$1; shift
  env "$@" timeout -k 10 120 python bench.py --config ${CFG:-3} --steps 20 --warmup 5 --no-cpu-baseline --no-strong --no-host-path --no-config4 --alt-math 0 > gpurun_out/${T}_$name.json 2> gpurun_out/${T}_$name.err || { tail -5 gpurun_out/${T}_$name.err; exit 1; }
  python -c "import json,sys; d=json.loads(open('gpurun_out/${T}_$name.json').read().splitlines()[-1]); print('$name', d['ms_per_step'], {k: d['kernel_ms'].get(k) for k in ('col2im','offset_bwd','offset_fwd')})"
}
for rep in 1 2; do
  for c in 3 4; do
    CFG=$c run cur_c${c}_$rep DCN_DUMMY=0
    CFG=$c run r03_c${c}_$rep DCN_LIB=tools/alt/alt0/libdcn.so DCN_FWD_WS=0 DCN_DW_WS=0
    for a in k5u4g k5u6 k5u8; do CFG=$c run ${a}_c${c}_$rep DCN_LIB=tools/alt/$a/libdcn.so; done
  done
done
echo k5 done
