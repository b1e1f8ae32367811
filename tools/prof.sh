#!/bin/bash
# rocprofv3 kernel stats of a short bench run. Usage: tools/prof.sh TAG [DCN_EXP]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
[ -n "$2" ] && export DCN_EXP="$2"
timeout -k 10 420 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$1 -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-strong > gpurun_out/prof_$1.log 2>&1 && echo "prof done"
