#!/bin/bash
# r03: bf16 fused forward (dcn_fused_bf16.hip) — its GPU parity tests, then config-4 benches
# per forward schedule (1 unfused, 2 fused + columns, 3 fused without columns) × DCN_EXP slot 0
# (VARIANTS="path_exp ...").
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${TAG:-fb1}
if [ "$1" != "--no-tests" ]; then
  timeout -k 10 300 python -u -m pytest tests/test_gpu_fused_bf16.py -x -q -rf --timeout 120 --timeout-method thread > gpurun_out/pytest_$T.log 2>&1; rc=$?
  tail -15 gpurun_out/pytest_$T.log
  [ $rc -eq 0 ] || exit $rc
fi
for v in ${VARIANTS:-1_0 2_0 3_0 1_0 2_0 3_0}; do
  set -- ${v/_/ }
  DCN_EXP=$2 timeout -k 10 120 python bench.py --config 4 --steps 20 --warmup 5 --no-cpu-baseline --no-host-path --no-strong --fwd-path $1 > gpurun_out/b4_${T}_$1_$2.json 2> gpurun_out/b4_${T}_$1_$2.err || { tail -5 gpurun_out/b4_${T}_$1_$2.err; exit 1; }
  python3 tools/kms.py gpurun_out/b4_${T}_$1_$2.json "path $1 exp $2"
done
