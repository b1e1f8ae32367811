#!/bin/bash
# r03: K5 flat batch stream — bitwise A/B against tools/prevlib, parity, variant timings.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
DCN_LIB=tools/prevlib/libdcn.so DCN_GEMM_BACKEND=hipblaslt timeout -k 10 300 python tools/ab_bitwise.py dump /tmp/ab_prev.npz > gpurun_out/ab_prev.log 2>&1 && \
DCN_GEMM_BACKEND=hipblaslt timeout -k 10 300 python tools/ab_bitwise.py dump /tmp/ab_new.npz > gpurun_out/ab_new.log 2>&1 && \
python tools/ab_bitwise.py cmp /tmp/ab_prev.npz /tmp/ab_new.npz > gpurun_out/ab_cmp.log 2>&1; rc=$?
grep -v "bitwise equal" gpurun_out/ab_cmp.log | tail -5
[ -s /tmp/ab_new.npz ] || { tail -20 gpurun_out/ab_new.log; exit 1; }
for v in 1 2; do
  DCN_EXP=$v timeout -k 10 400 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_bf16.py -q -x --timeout 200 --timeout-method thread 2>&1 | tail -1 || exit 1
done
CONFIG=3 bash tools/ab_cfg.sh k5s3 0 1 2 0 1 2 && CONFIG=4 bash tools/ab_cfg.sh k5s4 0 1 2 0 1 2
for l in prev new; do
  lib=$PWD/jittor-dcn_amd/lib/libdcn.so; [ $l = prev ] && lib=$PWD/tools/prevlib/libdcn.so
  for c in 3 4; do
    DCN_LIB=$lib timeout -k 10 240 python bench.py --config $c --steps 20 --warmup 5 --no-cpu-baseline --no-host-path --no-strong > gpurun_out/libab_$l.json 2> gpurun_out/libab_$l.err || { tail -5 gpurun_out/libab_$l.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/libab_$l.json'));k=d['kernel_ms'];print('c$c', '$l', d['ms_per_step'], k.get('col2im'))"
  done
done
