#!/bin/bash
# r03: bf16 fused forward (dcn_fused_bf16.hip) — its GPU parity tests, then config-4 benches
# per forward schedule (1 unfused, 2 fused + columns, 3 fused without columns).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${TAG:-fb1}
timeout -k 10 300 python -u -m pytest tests/test_gpu_fused_bf16.py -x -q -rf --timeout 120 --timeout-method thread > gpurun_out/pytest_$T.log 2>&1; rc=$?
tail -15 gpurun_out/pytest_$T.log
[ $rc -eq 0 ] || exit $rc
for p in 1 2 3 1 2 3; do
  timeout -k 10 120 python bench.py --config 4 --steps 20 --warmup 5 --no-cpu-baseline --no-host-path --no-strong --fwd-path $p > gpurun_out/b4_${T}_$p.json 2> gpurun_out/b4_${T}_$p.err || { tail -5 gpurun_out/b4_${T}_$p.err; exit 1; }
  python3 tools/kms.py gpurun_out/b4_${T}_$p.json "path $p"
done
