#!/bin/bash
# A/B of the current libdcn against tools/prevlib/libdcn.so (the previous commit's build):
# config-3 and config-4 steps, interleaved, bench kernel timings. Usage: tools/r03_libab.sh [REPS]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for rep in $(seq ${1:-2}); do
  for c in 3 4; do
    for l in prev new; do
      lib=$PWD/jittor-dcn_amd/lib/libdcn.so; [ $l = prev ] && lib=$PWD/tools/prevlib/libdcn.so
      DCN_LIB=$lib timeout -k 10 240 python bench.py --config $c --steps 20 --warmup 5 --no-cpu-baseline --no-host-path --no-strong > gpurun_out/libab_$l.json 2> gpurun_out/libab_$l.err || { tail -5 gpurun_out/libab_$l.err; exit 1; }
      python -c "import json;d=json.load(open('gpurun_out/libab_$l.json'));k=d['kernel_ms'];print('c$c', '$l', d['ms_per_step'], {x:k[x] for x in k if 'gemm_fwd' in x or 'bias' in x})"
    done
  done
done
