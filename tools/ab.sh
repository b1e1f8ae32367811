#!/bin/bash
# A/B of build or environment variants on one box, interleaved: tools/ab.sh TAG V1 V2 ...
# Each variant is a space-separated list of VAR=value settings for bench.py's process, e.g.
# "DCN_DW_GEMM=1" (the vendor ∂W GEMM), "DCN_LIB=tools/alt/r04/libdcn.so" (an older build,
# git-ignored), or "-" for the defaults. REPS rounds (default 2) of one short bench per
# variant; CONFIG (default 4) picks the BASELINE config; BENCH_EXTRA adds bench.py flags.
# Prints ms_per_step and the per-kernel-class HIP-event times of every run.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=$1
shift
for rep in $(seq 1 "${REPS:-2}"); do
  i=0
  for v in "$@"; do
    i=$((i + 1))
    envs=()
    [ "$v" != "-" ] && read -r -a envs <<< "$v"
    out=gpurun_out/ab_${TAG}_${i}_${rep}
    env "${envs[@]}" timeout -k 10 240 python bench.py --config "${CONFIG:-4}" --steps 10 --warmup 3 \
      --no-cpu-baseline --no-strong --no-host-path --no-config4 --no-extra-configs --alt-math 0 \
      ${BENCH_EXTRA} > $out.json 2> $out.err || { echo "variant '$v' failed"; tail -5 $out.err; exit 1; }
    python3 -c "
import json; d = json.load(open('$out.json')); k = d['kernel_ms']
print('rep $rep', repr('$v'), d['ms_per_step'], {x: round(y, 4) for x, y in k.items()})"
  done
done
