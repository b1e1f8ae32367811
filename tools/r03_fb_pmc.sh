#!/bin/bash
# r03: SQ counters of the bf16 fused forward at config 4 (fwd path $FP, DCN_EXP values given).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${TAG:-fbp}
FP=${FP:-3}
P1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES"
P2="SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_LEVEL_WAVES"
P3="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL"
for e in "$@"; do
  i=0
  for P in "$P1" "$P2" "$P3"; do
    i=$((i+1))
    DCN_EXP=$e timeout -k 10 120 rocprofv3 --pmc $P --kernel-trace -d gpurun_out/${T}_e${e}_p$i -o run --output-format csv -- python3 bench.py --config 4 --fwd-path $FP --steps 2 --warmup 1 --no-cpu-baseline --no-strong --no-host-path > gpurun_out/${T}_e${e}_p$i.log 2>&1 || { tail -5 gpurun_out/${T}_e${e}_p$i.log; exit 1; }
  done
  echo "== DCN_EXP=$e"
  python3 tools/pmc_table.py gpurun_out/${T}_e${e}_p1 gpurun_out/${T}_e${e}_p2 gpurun_out/${T}_e${e}_p3 --match=${MATCH:-fwd_fused_bf16}
done
