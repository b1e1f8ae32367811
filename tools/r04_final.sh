#!/bin/bash
# r04 round-end evidence on one box: the GPU suite, smoke, the many-launch determinism check,
# the default bench line (config 3 headline + the config-4 leg + CPU baseline), rocprofv3 kernel
# stats for configs 3 and 4, and the HBM PMC passes for both. Stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${1:-r04f}
B="--steps 5 --warmup 2 --no-cpu-baseline --no-strong --no-host-path"
echo "== pytest -m gpu" && \
timeout -k 10 600 python -u -m pytest tests -m gpu -q -rf --timeout 120 --timeout-method thread > gpurun_out/${T}_pytest_gpu.log 2>&1 || { tail -30 gpurun_out/${T}_pytest_gpu.log; exit 1; }
tail -2 gpurun_out/${T}_pytest_gpu.log
echo "== smoke" && timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" && \
echo "== launch_diag" && \
timeout -k 10 300 python -u tools/launch_diag.py --reps 200 --reps3 40 --out gpurun_out/${T}_launch_diag.json > gpurun_out/${T}_launch_diag.log 2>&1 || { tail -3 gpurun_out/${T}_launch_diag.log | cut -c1-600; exit 1; }
echo "launch_diag ok" && \
echo "== bench" && \
timeout -k 10 480 python bench.py > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err && cat gpurun_out/${T}_bench.json | cut -c1-1500 && \
echo "== rocprofv3 config 3" && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_prof3 -o run --output-format csv -- python3 bench.py $B --no-config4 --alt-math 0 > gpurun_out/${T}_prof3.log 2>&1 && \
echo "== rocprofv3 config 4" && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_prof4 -o run --output-format csv -- python3 bench.py $B --no-config4 --config 4 > gpurun_out/${T}_prof4.log 2>&1 && \
echo "== PMC config 3" && bash tools/pmc_pass.sh ${T}c3 && \
echo "== PMC config 4" && BENCH_ARGS="--config 4" bash tools/pmc_pass.sh ${T}c4 && \
echo "== bitwise dumps against r03's K5 / offset conv (tools/alt/alt0), GEMM choice pinned, bf16 ∂columns on hipBLASLt in both" && \
PIN="DCN_GEMM_BACKEND=hipblaslt DCN_GEMM_CANDIDATES=1" && \
env $PIN DCN_LIB=tools/alt/alt0/libdcn.so timeout -k 10 300 python tools/ab_bitwise.py dump /tmp/ab_a.npz > gpurun_out/${T}_ab.log 2>&1 && \
env $PIN DCN_DCOL_GEMM=1 timeout -k 10 300 python tools/ab_bitwise.py dump /tmp/ab_b.npz >> gpurun_out/${T}_ab.log 2>&1 && \
{ timeout -k 10 120 python tools/ab_bitwise.py cmp /tmp/ab_a.npz /tmp/ab_b.npz >> gpurun_out/${T}_ab.log 2>&1; grep -v "bitwise equal" gpurun_out/${T}_ab.log | tail -6; } && \
echo "final evidence done"
