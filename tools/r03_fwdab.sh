#!/bin/bash
# Offset-conv forward change check: its parity tests, a bitwise dump against the previous
# build (tools/prevlib), then interleaved config-3/4 timings. Usage: tools/r03_fwdab.sh [REPS]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_bf16.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/fwdab_pytest.log 2>&1 || { tail -30 gpurun_out/fwdab_pytest.log; exit 1; }
tail -3 gpurun_out/fwdab_pytest.log
DCN_LIB=$PWD/tools/prevlib/libdcn.so timeout -k 10 300 python tools/ab_bitwise.py dump gpurun_out/fwdab_a.npz > gpurun_out/fwdab_dump_a.log 2>&1 || { tail -20 gpurun_out/fwdab_dump_a.log; exit 1; }
timeout -k 10 300 python tools/ab_bitwise.py dump gpurun_out/fwdab_b.npz > gpurun_out/fwdab_dump_b.log 2>&1 || { tail -20 gpurun_out/fwdab_dump_b.log; exit 1; }
python tools/ab_bitwise.py cmp gpurun_out/fwdab_a.npz gpurun_out/fwdab_b.npz | grep -E "_off |ALL|differ"
rm -f gpurun_out/fwdab_a.npz gpurun_out/fwdab_b.npz
for rep in $(seq ${1:-2}); do
  for c in 3 4; do
    for l in prev new; do
      lib=$PWD/jittor-dcn_amd/lib/libdcn.so; [ $l = prev ] && lib=$PWD/tools/prevlib/libdcn.so
      DCN_LIB=$lib timeout -k 10 240 python bench.py --config $c --steps 20 --warmup 5 --no-cpu-baseline --no-host-path --no-strong > gpurun_out/fwdab_$l.json 2> gpurun_out/fwdab_$l.err || { tail -5 gpurun_out/fwdab_$l.err; exit 1; }
      python -c "import json;d=json.load(open('gpurun_out/fwdab_$l.json'));k=d['kernel_ms'];print('c$c', '$l', d['ms_per_step'], {x:k[x] for x in k if 'offset' in x or 'xpose' in x})"
    done
  done
done
