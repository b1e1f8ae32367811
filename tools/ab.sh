#!/bin/bash
# A/B development knobs on the GPU: GPU parity tests with the defaults, then one short
# bench per DCN_EXP variant. Usage: tools/ab.sh TAG "v1" "v2" ...
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=$1; shift
mkdir -p gpurun_out
timeout -k 10 420 python -m pytest tests -m gpu -q -x > gpurun_out/ab_pytest_$TAG.log 2>&1; rc=$?
tail -3 gpurun_out/ab_pytest_$TAG.log
[ $rc -eq 0 ] || { echo "pytest rc=$rc"; tail -40 gpurun_out/ab_pytest_$TAG.log; exit $rc; }
for v in "$@"; do
  DCN_EXP="$v" timeout -k 10 240 python bench.py --steps 10 --warmup 3 --no-cpu-baseline $BENCH_ARGS > gpurun_out/ab_${TAG}_$v.json 2> gpurun_out/ab_${TAG}_$v.err || { echo "bench $v failed"; tail -5 gpurun_out/ab_${TAG}_$v.err; exit 1; }
  python -c "
import json,sys; d=json.load(open('gpurun_out/ab_${TAG}_$v.json'))
print('$v', d['ms_per_step'], {k: round(v,3) for k,v in d['kernel_ms'].items()})"
done
