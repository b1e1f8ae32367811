#!/bin/bash
# r04: many-launch determinism of the shipped kernels (tools/launch_diag.py), the GPU suite,
# smoke, the default bench (config 3 headline + the config-4 leg) and its rocprofv3 stats.
# Every GPU step has its own time limit; the chain stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-r04a}
echo "== fused bf16 parity first (new kernels, short limit)" && \
timeout -k 10 240 python -u -m pytest tests/test_gpu_fused_bf16.py -x -q --timeout 100 --timeout-method thread > gpurun_out/fused_first_$TAG.log 2>&1; rc=$?
tail -4 gpurun_out/fused_first_$TAG.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || { echo "fused tests aborted rc=$rc"; exit $rc; }
echo "== launch_diag" && \
timeout -k 10 300 python -u tools/launch_diag.py --reps ${REPS:-200} --out gpurun_out/launch_diag_$TAG.json > gpurun_out/launch_diag_$TAG.log 2>&1; rc=$?
tail -3 gpurun_out/launch_diag_$TAG.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || { echo "launch_diag aborted rc=$rc"; exit $rc; }
echo "== pytest -m gpu" && \
timeout -k 10 600 python -u -m pytest tests -m gpu -q -rf --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_$TAG.log 2>&1; rc=$?
tail -25 gpurun_out/pytest_gpu_$TAG.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || { echo "pytest aborted rc=$rc"; exit $rc; }
echo "== smoke" && \
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" && \
echo "== bench" && \
timeout -k 10 420 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err && \
cat gpurun_out/bench_$TAG.json && \
echo "== rocprofv3" && \
timeout -k 10 420 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-strong --no-host-path --alt-math 0 > gpurun_out/prof_$TAG.log 2>&1 && \
echo "done"
