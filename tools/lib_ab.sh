#!/bin/bash
# A/B of alternative libdcn builds (LIBS="name ...", jittor-dcn_amd/lib/libdcn_<name>.so;
# "base" = libdcn.so) x DCN_EXP variants (EXPS), math mode MATH, bench kernel timings.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for rep in 1 2; do
for l in ${LIBS:-base}; do
  lib=jittor-dcn_amd/lib/libdcn_$l.so; [ "$l" = base ] && lib=jittor-dcn_amd/lib/libdcn.so
  for e in ${EXPS:-0}; do
    DCN_LIB=$PWD/$lib DCN_EXP=$e timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --math ${MATH:-6} > gpurun_out/libab.json 2>gpurun_out/libab.err || { tail -5 gpurun_out/libab.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/libab.json'));k=d['kernel_ms'];print('$l', '$e', d['ms_per_step'], {x:k[x] for x in k if 'gemm' in x})"
  done
done
done
