#!/bin/bash
# r04: confirmation of the committed tree on one box: pytest -m gpu, smoke(), the default bench line (no CPU baseline).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -q -rf --timeout 120 --timeout-method thread > gpurun_out/r04c_pytest_gpu.log 2>&1 || { tail -30 gpurun_out/r04c_pytest_gpu.log; exit 1; }
tail -2 gpurun_out/r04c_pytest_gpu.log
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" && \
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/r04c_bench.json 2> gpurun_out/r04c_bench.err && python -c "import json; d=json.loads(open('gpurun_out/r04c_bench.json').read().splitlines()[-1]); print('c3', d['ms_per_step'], d['value'], 'c4', d['config4']['ms_per_step'], d['config4']['kernel_ms'])"
