#!/bin/bash
# r03: fused-forward corruption diagnosis (tools/fused_diag), bitwise A/B of the bins
# rewrite against the previous build, GPU tests, rocprofv3 stats of a config-3 step.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
echo "== fused_diag" && \
timeout -k 10 240 ./tools/fused_diag/fused_diag 8 > gpurun_out/fused_diag3.log 2>&1; rc=$?
grep -E "SUMMARY|errors by|nondeterminism by" gpurun_out/fused_diag3.log
[ $rc -eq 0 ] || { echo "fused_diag rc=$rc"; exit $rc; }
echo "== ab prev" && \
DCN_LIB=tools/prevlib/libdcn.so timeout -k 10 300 python tools/ab_bitwise.py dump /tmp/ab_prev.npz > gpurun_out/ab_prev.log 2>&1 && \
echo "== ab new" && \
timeout -k 10 300 python tools/ab_bitwise.py dump /tmp/ab_new.npz > gpurun_out/ab_new.log 2>&1 && \
python tools/ab_bitwise.py cmp /tmp/ab_prev.npz /tmp/ab_new.npz > gpurun_out/ab_cmp.log 2>&1; rc=$?
cat gpurun_out/ab_cmp.log
echo "== pytest -m gpu" && \
timeout -k 10 420 python -u -m pytest tests -m gpu -q -rf -x --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_r03b.log 2>&1; rc=$?
tail -15 gpurun_out/pytest_gpu_r03b.log
[ $rc -eq 0 ] || { echo "pytest rc=$rc"; exit $rc; }
echo "== rocprofv3" && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r03b -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-strong --no-host-path > gpurun_out/prof_r03b.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof4_r03b -o run --output-format csv -- python3 bench.py --config 4 --steps 5 --warmup 2 --no-cpu-baseline --no-strong --no-host-path > gpurun_out/prof4_r03b.log 2>&1 && \
echo done
