#!/bin/bash
# Short benches per DCN_EXP variant without the test suite. Usage: CONFIG=N tools/ab_cfg.sh TAG v1 v2 ...
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=$1; shift
mkdir -p gpurun_out
for v in "$@"; do
  DCN_EXP="$v" timeout -k 10 240 python bench.py --config ${CONFIG:-3} --steps 20 --warmup 5 --no-cpu-baseline --no-host-path --no-strong > gpurun_out/abc_${TAG}_$v.json 2> gpurun_out/abc_${TAG}_$v.err || { echo "bench $v failed"; tail -5 gpurun_out/abc_${TAG}_$v.err; exit 1; }
  python -c "
import json,sys; d=json.load(open('gpurun_out/abc_${TAG}_$v.json'))
print('c${CONFIG:-3}', '$v', d['ms_per_step'], {k: round(v,3) for k,v in d['kernel_ms'].items()})"
done
