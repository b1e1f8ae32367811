#!/bin/bash
# MFMA utilisation counters per kernel (MI355X_MICROARCH.md "Per-instruction
# cycle constants": SQ_VALU_MFMA_BUSY_CYCLES counts matrix-pipe cycles, GRBM_GUI_ACTIVE the GPU's
# active cycles summed over the 8 XCDs). One pass (3 SQ + 1 GRBM slots), kernel trace only, no
# other trace domain. Usage: tools/pmc_mfma.sh TAG [bench.py flags, e.g. --config 4]
# Summarise with tools/mfma_summary.py (gpu.sh mfma3 / mfma4 / mfma5 do both).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=$1
shift
timeout -s KILL 240 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE \
  --kernel-trace -d gpurun_out/mfma_$TAG -o run --output-format csv -- \
  python3 bench.py --steps 3 --warmup 2 --no-cpu-baseline --no-strong --no-host-path --no-config4 \
  --no-extra-configs --alt-math 0 "$@" > gpurun_out/mfma_$TAG.log 2>&1 && echo "mfma pass done"
