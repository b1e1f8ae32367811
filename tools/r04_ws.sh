#!/bin/bash
# r04: the warp-specialised bf16 fused forward (fwd_fused_bf16_ws) — its parity tests, the
# many-launch determinism diag, then config-4 benches against the r03 kernel (DCN_FWD_WS=0,
# temporary A/B switch) interleaved, and the rocprofv3 kernel stats of the new one.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${1:-ws1}
echo "== pytest (fused bf16, bf16, ednet)" && \
timeout -k 10 400 python -u -m pytest tests/test_gpu_fused_bf16.py tests/test_gpu_bf16.py tests/test_gpu_ednet.py -q -x --timeout 120 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1; rc=$?
tail -5 gpurun_out/${T}_pytest.log
[ $rc -eq 0 ] || { echo "pytest rc=$rc"; exit $rc; }
echo "== launch_diag" && \
timeout -k 10 240 python -u tools/launch_diag.py --reps ${REPS:-100} --reps3 10 --out gpurun_out/${T}_diag.json > gpurun_out/${T}_diag.log 2>&1; rc=$?
tail -2 gpurun_out/${T}_diag.log | cut -c1-600
[ $rc -eq 0 ] || [ $rc -eq 1 ] || { echo "diag rc=$rc"; exit $rc; }
for v in 0 1 0 1; do
  DCN_FWD_WS=$v timeout -k 10 200 python bench.py --config 4 --steps 30 --warmup 5 --no-cpu-baseline --no-strong --no-host-path > gpurun_out/${T}_b4_$v.json 2> gpurun_out/${T}_b4_$v.err || { tail -5 gpurun_out/${T}_b4_$v.err; exit 1; }
  python tools/kms.py gpurun_out/${T}_b4_$v.json 2>/dev/null | head -3 || head -c 600 gpurun_out/${T}_b4_$v.json
done
echo "== rocprofv3 config 4" && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_prof4 -o run --output-format csv -- python3 bench.py --config 4 --steps 10 --warmup 3 --no-cpu-baseline --no-strong --no-host-path > gpurun_out/${T}_prof4.log 2>&1 && \
echo done
