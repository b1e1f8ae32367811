#!/bin/bash
# HBM traffic counters for every libdcn kernel of a short bench run (MI355X_MICROARCH.md
# "HBM" section): FETCH_SIZE and WRITE_SIZE in separate passes (TCC slots), kernel trace
# only; BENCH_ARGS passes extra bench.py flags (--config 4). Summarise with tools/pmc_summary.py.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=${1:-r01}
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/pmc_fetch_$TAG -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-strong --no-host-path --no-config4 --no-extra-configs --alt-math 0 ${BENCH_ARGS} > gpurun_out/pmc_fetch_$TAG.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d gpurun_out/pmc_write_$TAG -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-strong --no-host-path --no-config4 --no-extra-configs --alt-math 0 ${BENCH_ARGS} > gpurun_out/pmc_write_$TAG.log 2>&1 && \
echo "pmc done"
