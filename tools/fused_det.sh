# run-to-run / fused-vs-unfused determinism probes
set -o pipefail
for v in ${FD_VARIANTS:-0}; do
  DCN_EXP=$v timeout -k 10 200 python -u tools/fused_det.py > gpurun_out/fdv$v.log 2>&1 || exit 1
  echo "== $v"; grep -v amdgpu.ids gpurun_out/fdv$v.log | grep "u2 f\|run-to-run\|out: frac"
done
if [ -n "$F32" ]; then timeout -k 10 200 python -u tools/det_f32.py > gpurun_out/det_f32.log 2>&1 || exit 1; grep -v amdgpu.ids gpurun_out/det_f32.log; fi
