#!/bin/bash
# dma_probe timings (every mode, rings of 4 and 3 slots) and, with PMC=1, counter passes over
# the dw / l2 / stream modes. Run on the GPU box from the repo root (the binary is built here:
# hipcc --offload-arch=gfx950 -O3 -o tools/dma_probe/dma_probe tools/dma_probe/dma_probe.hip).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
B=tools/dma_probe/dma_probe
OUT=gpurun_out/dma_probe_${1:-r06}.jsonl
: > "$OUT"
for R in 4 3; do
  for m in dw l2 contig unique stream stream1 dw2; do
    timeout -k 10 60 $B $m $R 20 >> "$OUT" || exit 1
  done
done
cat "$OUT"
[ "${PMC:-0}" = 1 ] || exit 0
timeout -k 10 60 rocprofv3 --list-avail > gpurun_out/dma_probe_avail.txt 2>&1 || true
pass() {  # NAME COUNTERS...: one counter pass over mode $m; a kill ends the script
  local name=$1; shift
  timeout -s KILL 60 rocprofv3 --pmc "$@" --kernel-trace -d gpurun_out/dmap_${name}_$m -o run --output-format csv -- $B $m 4 5 > gpurun_out/dmap_${name}_$m.log 2>&1
  local rc=$?
  if [ $rc = 137 ] || [ $rc = 124 ]; then echo "pass $name $m killed"; exit 1; fi
  echo "pass $name $m rc=$rc"
}
for m in dw l2 stream; do
  pass fetch FETCH_SIZE
  pass tcc TCC_HIT_sum TCC_MISS_sum
  pass tcp TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum TCP_TOTAL_CACHE_ACCESSES_sum
  pass ta TA_BUSY_avr TA_BUFFER_WAVEFRONTS_sum
  pass sq GRBM_GUI_ACTIVE SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAVE_CYCLES
done
echo "pmc done"
