#!/bin/bash
# r03: the bf16 GPU suites (fused forward / no-column path, and the bf16 path whose
# config-4 tests run the DCN_FWD_AUTO schedule), then config-4 A/B per forward schedule.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${TAG:-fbc}
timeout -k 10 400 python -u -m pytest tests/test_gpu_fused_bf16.py tests/test_gpu_bf16.py -x -q -rf --timeout 200 --timeout-method thread > gpurun_out/pytest_$T.log 2>&1; rc=$?
tail -5 gpurun_out/pytest_$T.log
[ $rc -eq 0 ] || { grep -E "Error|assert" gpurun_out/pytest_$T.log | head -20; exit $rc; }
VARIANTS="${VARIANTS:-1_0 2_0 3_0 0_0 1_0 2_0 3_0 0_0}" TAG=$T bash tools/r03_fusedbf16.sh --no-tests
