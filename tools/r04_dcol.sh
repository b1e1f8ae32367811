#!/bin/bash
# r04: the bf16 ∂columns on dcol_bf16 (short-K streaming kernel) against the vendor GEMM
# (DCN_DCOL_GEMM=1, same build; ALT='path/libdcn.so ...' adds other builds): bf16 parity, then
# config-4 A/B (bench.py, HIP events) and a
# rocprofv3 kernel-stats pass. Stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${1:-dcol}
timeout -k 10 300 python -u -m pytest tests/test_gpu_bf16.py tests/test_gpu_fused_bf16.py -x -q --timeout 120 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1 || { tail -30 gpurun_out/${T}_pytest.log; exit 1; }
echo "parity: $(tail -1 gpurun_out/${T}_pytest.log)"
run() {  # name env...
  local name=$1; shift
  env "$@" timeout -k 10 120 python bench.py --config 4 --steps 20 --warmup 5 --no-cpu-baseline --no-strong --no-host-path --no-config4 > gpurun_out/${T}_$name.json 2> gpurun_out/${T}_$name.err || { tail -5 gpurun_out/${T}_$name.err; exit 1; }
  python -c "import json,sys; d=json.loads(open('gpurun_out/${T}_$name.json').read().splitlines()[-1]); print('$name', d['ms_per_step'], {k: d['kernel_ms'].get(k) for k in ('gemm_dcol','col2im','gemm_dw')})"
}
for rep in 1 2 3; do
  run new_$rep DCN_DUMMY=0 || exit 1
  for a in $ALT; do run $(basename $(dirname $a))_$rep DCN_LIB=$a || exit 1; done
  run gemm_$rep DCN_DCOL_GEMM=1 || exit 1
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_prof4 -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-strong --no-host-path --no-config4 --config 4 > gpurun_out/${T}_prof4.log 2>&1 || { tail -5 gpurun_out/${T}_prof4.log; exit 1; }
grep -i "dcol" gpurun_out/${T}_prof4/run_kernel_stats.csv | cut -c1-200
echo dcol done
