#!/bin/bash
# GPU suite, then short benches of config 4 (bf16) and config 3 (fp32).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-chk}
timeout -k 10 420 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_$TAG.log
[ $rc -eq 0 ] || { grep -E "Error|error|FAILED|assert" gpurun_out/pytest_$TAG.log | head -30; exit $rc; }
for c in ${CONFIGS:-4 3}; do
  timeout -k 10 300 python bench.py --config $c --steps 20 --warmup 5 --no-cpu-baseline --no-host-path > gpurun_out/bench_${TAG}_c$c.json 2> gpurun_out/bench_${TAG}_c$c.err || { tail -5 gpurun_out/bench_${TAG}_c$c.err; exit 1; }
  python -c "
import json; d=json.load(open('gpurun_out/bench_${TAG}_c$c.json'))
print('config $c', d['ms_per_step'], d['value'], {k: round(v,3) for k,v in d['kernel_ms'].items()}, 'K1 frac', d['roofline']['frac'])"
done
