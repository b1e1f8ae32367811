#!/bin/bash
# Host-pointer API: GPU tests, then the PCIe-inclusive rate at config 3 under staging /
# copy-thread / reuse variants (tools/host_rate.py).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_host.py -q -x --timeout 120 --timeout-method thread > gpurun_out/host_pytest.log 2>&1; rc=$?
tail -3 gpurun_out/host_pytest.log
[ $rc -eq 0 ] || { tail -40 gpurun_out/host_pytest.log; exit $rc; }
for v in "HOST_REUSE=0" "HOST_REUSE=1" "DCN_HOST_STAGING=1 DCN_HOST_THREADS=8" "DCN_HOST_STAGING=1 DCN_HOST_THREADS=16"; do
  env $v timeout -k 10 200 python tools/host_rate.py || exit 1
done
