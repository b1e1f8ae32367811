#!/bin/bash
# r03: every GPU test, rocprofv3 kernel stats at configs 3 and 4 (K5 boundary partials),
# then the host-pointer rates (tools/host_rate.py: chunk sweep, 4-module stack).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${TAG:-r03k}
echo "== pytest -m gpu" && \
timeout -k 10 600 python -u -m pytest tests -m gpu -q -rf -x --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu_$T.log 2>&1; rc=$?
tail -8 gpurun_out/pytest_gpu_$T.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/pytest_gpu_$T.log | head -30; exit $rc; }
echo "== prof" && \
bash tools/prof_cfg.sh ${T}_c3 3 > gpurun_out/kstats_${T}_c3.txt && \
bash tools/prof_cfg.sh ${T}_c4 4 > gpurun_out/kstats_${T}_c4.txt && \
grep -iE "col2im|fold|bins|total" gpurun_out/kstats_${T}_c3.txt gpurun_out/kstats_${T}_c4.txt | head -30 && \
echo "== host" && \
timeout -k 10 300 python -u tools/host_rate.py --chunks ${CHUNKS:-1,4,0} --steps 4 && \
timeout -k 10 300 python -u tools/host_rate.py --chunks 1,0 --stack 4 --steps 3
