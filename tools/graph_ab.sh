#!/bin/bash
# Eager vs HIP-graph replay of the bench step (bench.py --graph), configs 3, 4 and 1.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
set -o pipefail
for c in 3 4 1; do for gr in 0 1 0 1; do
  timeout -k 10 120 python bench.py --config $c --steps 20 --warmup 5 --no-cpu-baseline --alt-math 0 --graph $gr > gpurun_out/gr_${c}_$gr.json || exit 1
  python -c "import json; d=json.load(open('gpurun_out/gr_${c}_$gr.json')); print($c, $gr, d['ms_per_step'], d['launch'])"
done; done
