#!/bin/bash
# rocprofv3 kernel stats for several DCN_EXP variants. Usage: tools/prof_exp.sh TAG v1 v2 ...
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=$1; shift
mkdir -p gpurun_out
for v in "$@"; do
  DCN_EXP="$v" timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "gpurun_out/px_${TAG}_$v" -o run \
    --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-strong --no-host-path ${BENCH_ARGS} \
    > "gpurun_out/px_${TAG}_$v.log" 2>&1 || { echo "variant $v failed"; exit 1; }
done
echo "prof_exp done"
