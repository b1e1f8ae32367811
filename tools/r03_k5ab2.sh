#!/bin/bash
# r03: K5 packed-math rewrite — bitwise A/B against the previous build (tools/prevlib), then
# variant timings (DCN_EXP slot 0) at configs 3 and 4.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
DCN_LIB=tools/prevlib/libdcn.so timeout -k 10 300 python tools/ab_bitwise.py dump /tmp/ab_prev.npz > gpurun_out/ab_prev.log 2>&1 && \
timeout -k 10 300 python tools/ab_bitwise.py dump /tmp/ab_new.npz > gpurun_out/ab_new.log 2>&1 && \
python tools/ab_bitwise.py cmp /tmp/ab_prev.npz /tmp/ab_new.npz > gpurun_out/ab_cmp.log 2>&1; rc=$?
tail -3 gpurun_out/ab_cmp.log
[ $rc -eq 0 ] || { cat gpurun_out/ab_cmp.log; tail -20 gpurun_out/ab_new.log; exit $rc; }
CONFIG=3 bash tools/ab_cfg.sh k5p3 0 2 1 0 2 1 && \
CONFIG=4 bash tools/ab_cfg.sh k5p4 0 2 1 0 2 1
