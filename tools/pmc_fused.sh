#!/bin/bash
# SQ counter passes over a short bench with the fused forward (DCN_FWD_FUSED); each pass its
# own run (tools/pmc_table.py gpurun_out/pmcf_1 gpurun_out/pmcf_2 --match=fwd_fused).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
i=0
for set in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" \
           "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_BUSY_CYCLES SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_SCA SQ_INSTS_VMEM"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $set --kernel-trace -d gpurun_out/pmcf_$i -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-strong --alt-math 0 --fwd-path ${FWD_PATH:-2} > gpurun_out/pmcf_$i.log 2>&1 || { echo "pass $i failed"; tail -3 gpurun_out/pmcf_$i.log; exit 1; }
done
echo done
