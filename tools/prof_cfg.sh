#!/bin/bash
# rocprofv3 kernel stats of a short bench at one config: tools/prof_cfg.sh TAG CONFIG [DCN_EXP]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
[ -n "$3" ] && export DCN_EXP="$3"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$1 -o run --output-format csv -- python3 bench.py --config $2 --steps 5 --warmup 2 --no-cpu-baseline --no-strong --no-host-path > gpurun_out/prof_$1.log 2>&1 && python3 tools/kstats.py gpurun_out/prof_$1
