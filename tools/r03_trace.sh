#!/bin/bash
# r03: memory-copy + kernel trace of the host-pointer path (tools/host_rate.py), and the
# K5 HBM / SQ counters at config 3 (separate --pmc passes, kernel trace only).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${TAG:-r03t}
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/htrace_$T -o run -- python3 tools/host_rate.py --chunks ${CHUNKS:-1,4} --steps 2 > gpurun_out/htrace_$T.log 2>&1 && \
cat gpurun_out/htrace_$T.log && \
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/pmc_fetch_$T -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-strong --no-host-path > gpurun_out/pmc_fetch_$T.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d gpurun_out/pmc_write_$T -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-strong --no-host-path > gpurun_out/pmc_write_$T.log 2>&1 && \
bash tools/pmc_sq.sh $T && echo "trace done"
