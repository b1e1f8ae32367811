#!/bin/bash
# A/B of alternative libdcn builds on the col2im / im2col / offset-conv times at configs 3 and
# 4 (LIBS="name ...": jittor-dcn_amd/lib/libdcn_<name>.so, "base" = libdcn.so), two rounds.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for rep in 1 2; do
for c in ${CONFIGS:-3 4}; do
for l in ${LIBS:-base}; do
  lib=jittor-dcn_amd/lib/libdcn_$l.so; [ "$l" = base ] && lib=jittor-dcn_amd/lib/libdcn.so
  DCN_LIB=$PWD/$lib timeout -k 10 200 python bench.py --config $c --steps 10 --warmup 3 --no-cpu-baseline --no-host-path --alt-math 0 > gpurun_out/libab.json 2>gpurun_out/libab.err || { tail -5 gpurun_out/libab.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/libab.json'));k=d['kernel_ms'];print('c$c', '$l', d['ms_per_step'], {x:k[x] for x in k if x in ('col2im','im2col','offset_fwd','offset_bwd')})"
done; done; done
