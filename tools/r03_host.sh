#!/bin/bash
# Host-pointer API on the box: its GPU tests (states, chunk pipeline, config-3 host path),
# then the PCIe-inclusive config-3 rate over chunk counts, single module and a 4-module stack.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_host.py tests/test_gpu_configs.py -v -x --timeout 200 --timeout-method thread > gpurun_out/host_pytest.log 2>&1; rc=$?
tail -5 gpurun_out/host_pytest.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/host_pytest.log | head -30; exit $rc; }
timeout -k 10 300 python -u tools/host_rate.py --chunks ${CHUNKS:-1,2,4,8,12,16,0} --steps 4 || exit 1
timeout -k 10 300 python -u tools/host_rate.py --chunks 1,0 --stack 4 --steps 2 || exit 1
