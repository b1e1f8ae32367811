#!/bin/bash
# Round-end evidence: GPU tests, smoke, bench (config 3 with CPU baseline; config 4 bf16),
# rocprofv3 kernel stats and HBM PMC passes. Usage: tools/round_profile.sh TAG
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=${1:-r01}
mkdir -p gpurun_out
bash tools/gpu_check.sh $TAG && \
timeout -k 10 300 python bench.py --config 4 --steps 20 --warmup 5 --no-cpu-baseline --no-strong --no-host-path > gpurun_out/bench4_$TAG.json 2> gpurun_out/bench4_$TAG.err && \
timeout -k 10 420 rocprofv3 --kernel-trace --stats -d gpurun_out/prof4_$TAG -o run --output-format csv -- python3 bench.py --config 4 --steps 5 --warmup 2 --no-cpu-baseline --no-strong --no-host-path > gpurun_out/prof4_$TAG.log 2>&1 && \
bash tools/pmc_pass.sh $TAG && \
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/pmc4_fetch_$TAG -o run --output-format csv -- python3 bench.py --config 4 --steps 2 --warmup 1 --no-cpu-baseline --no-strong --no-host-path > gpurun_out/pmc4_fetch_$TAG.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d gpurun_out/pmc4_write_$TAG -o run --output-format csv -- python3 bench.py --config 4 --steps 2 --warmup 1 --no-cpu-baseline --no-strong --no-host-path > gpurun_out/pmc4_write_$TAG.log 2>&1 && \
echo "round profile done"
