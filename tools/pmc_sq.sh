#!/bin/bash
# SQ instruction / stall counters per kernel (two 8-counter passes, kernel trace only).
# Usage: [P1="..."] [P2="..."] tools/pmc_sq.sh TAG [DCN_EXP]; summarise with tools/pmc_table.py.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
[ -n "$2" ] && export DCN_EXP="$2"
P1="${P1:-SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES}"
P2="${P2:-SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_LEVEL_WAVES}"
timeout -k 10 300 rocprofv3 --pmc $P1 --kernel-trace -d gpurun_out/sq1_$1 -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-strong --no-host-path --no-config4 --no-extra-configs --alt-math 0 ${BENCH_ARGS} > gpurun_out/sq1_$1.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc $P2 --kernel-trace -d gpurun_out/sq2_$1 -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-strong --no-host-path --no-config4 --no-extra-configs --alt-math 0 ${BENCH_ARGS} > gpurun_out/sq2_$1.log 2>&1 && \
echo "sq done"
