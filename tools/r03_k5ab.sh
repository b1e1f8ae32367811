#!/bin/bash
# r03: K5 variants (DCN_EXP slot 0) — GPU parity of the backward, then config 3 / 4 A/B.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in 0 2; do
  DCN_EXP=$v timeout -k 10 400 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_parity.py tests/test_gpu_bf16.py -q -x --timeout 200 --timeout-method thread > gpurun_out/k5ab_pytest_$v.log 2>&1 || { tail -30 gpurun_out/k5ab_pytest_$v.log; exit 1; }
  tail -1 gpurun_out/k5ab_pytest_$v.log
done
CONFIG=3 bash tools/ab_cfg.sh k5c3 1 0 2 3 4 1 0 2 && \
CONFIG=4 bash tools/ab_cfg.sh k5c4 1 0 2 3 4 1 0 2
