#!/bin/bash
# Gradient-exchange paths of bench.py on one GPU (a 1-rank RCCL group): torch.distributed
# with the grad-stream overlap, and libdcn's own communicator attached to the handle, for
# config 3 (fp32) and config 4 (bf16). Also prints the host CPU share the CPU baseline sees.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
python -c "import bench, json; print(json.dumps(bench.host_cpus()))" && \
for cfg in 3 4; do for comm in torch libdcn; do
  timeout -k 10 180 python bench.py --config $cfg --steps 10 --warmup 3 --no-cpu-baseline --alt-math 0 \
      --exchange --comm $comm > gpurun_out/exch_${cfg}_${comm}.json 2> gpurun_out/exch_${cfg}_${comm}.err || exit $?
  python -c "import json,sys; d=json.loads([l for l in open('gpurun_out/exch_${cfg}_${comm}.json') if l.startswith('{')][-1]); print($cfg, '$comm', d['ms_per_step'], d['config']['grad_allreduce'])" || exit 1
done; done
echo "exchange check done"
