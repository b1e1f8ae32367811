#!/bin/bash
# r03: bitwise A/B against the previous build, GPU tests, rocprofv3 stats (configs 3, 4),
# then the fused-forward XOR-checksum diagnosis
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-r03e}
echo "== ab" && \
DCN_LIB=tools/prevlib/libdcn.so timeout -k 10 300 python tools/ab_bitwise.py dump /tmp/ab_prev.npz > gpurun_out/ab_prev.log 2>&1 && \
timeout -k 10 300 python tools/ab_bitwise.py dump /tmp/ab_new.npz > gpurun_out/ab_new.log 2>&1 && \
python tools/ab_bitwise.py cmp /tmp/ab_prev.npz /tmp/ab_new.npz > gpurun_out/ab_cmp_$TAG.log 2>&1; rc=$?
tail -1 gpurun_out/ab_cmp_$TAG.log
echo "== pytest -m gpu" && \
timeout -k 10 480 python -u -m pytest tests -m gpu -q -rf --timeout 150 --timeout-method thread > gpurun_out/pytest_gpu_$TAG.log 2>&1; rc=$?
tail -5 gpurun_out/pytest_gpu_$TAG.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || { echo "pytest aborted rc=$rc"; exit $rc; }
echo "== rocprofv3" && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-strong > gpurun_out/prof_$TAG.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof4_$TAG -o run --output-format csv -- python3 bench.py --config 4 --steps 5 --warmup 2 --no-cpu-baseline --no-strong > gpurun_out/prof4_$TAG.log 2>&1 && \
echo "== bench" && \
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-strong > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err && \
timeout -k 10 300 python bench.py --config 4 --steps 20 --warmup 5 --no-cpu-baseline --no-strong > gpurun_out/bench4_$TAG.json 2> gpurun_out/bench4_$TAG.err && \
python3 -c "
import json
for f in ['gpurun_out/bench_$TAG.json','gpurun_out/bench4_$TAG.json']:
    d=json.loads(open(f).read().strip().splitlines()[-1])
    print(f, d['ms_per_step'], d['value'])
" && \
[ -n "$SKIP_DIAG" ] && { echo done; exit 0; }
echo "== fused_diag" && \
timeout -k 10 240 ./tools/fused_diag/fused_diag 5 > gpurun_out/fused_diag5.log 2>&1; rc=$?
grep -E "SUMMARY|XOR" gpurun_out/fused_diag5.log | head -30
exit $rc
