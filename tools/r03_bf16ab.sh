#!/bin/bash
# bf16 forward-GEMM layout change: bf16 parity tests, then interleaved config-4 steps against
# tools/prevlib. Usage: tools/r03_bf16ab.sh [REPS]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_bf16.py tests/test_gpu_host.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/bf16ab_pytest.log 2>&1 || { tail -30 gpurun_out/bf16ab_pytest.log; exit 1; }
tail -3 gpurun_out/bf16ab_pytest.log
DCN_LIB=$PWD/tools/prevlib/libdcn.so timeout -k 10 300 python tools/ab_bitwise.py dump gpurun_out/bf16ab_a.npz > gpurun_out/bf16ab_dump_a.log 2>&1 || { tail -20 gpurun_out/bf16ab_dump_a.log; exit 1; }
timeout -k 10 300 python tools/ab_bitwise.py dump gpurun_out/bf16ab_b.npz > gpurun_out/bf16ab_dump_b.log 2>&1 || { tail -20 gpurun_out/bf16ab_dump_b.log; exit 1; }
python tools/ab_bitwise.py cmp gpurun_out/bf16ab_a.npz gpurun_out/bf16ab_b.npz | grep -E "DIFFERS|ALL|differ" || true
rm -f gpurun_out/bf16ab_a.npz gpurun_out/bf16ab_b.npz
for rep in $(seq ${1:-3}); do
  for l in prev new; do
    lib=$PWD/jittor-dcn_amd/lib/libdcn.so; [ $l = prev ] && lib=$PWD/tools/prevlib/libdcn.so
    DCN_LIB=$lib timeout -k 10 240 python bench.py --config 4 --steps 30 --warmup 5 --no-cpu-baseline --no-host-path --no-strong > gpurun_out/bf16ab_$l.json 2> gpurun_out/bf16ab_$l.err || { tail -5 gpurun_out/bf16ab_$l.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/bf16ab_$l.json'));k=d['kernel_ms'];print('c4', '$l', d['ms_per_step'], {x:k[x] for x in k if x in ('gemm_fwd','bias_fwd','offset_bwd','offset_fwd')})"
  done
done
