#!/bin/bash
# K5 A/B at config 3 (BENCH_ARGS="--config 4" for config 4): r01 tile kernel vs the column
# sweep (batch prefetch U / ring prefetch D, DCN_EXP slots 10, 12, 13), then HBM PMC passes
# of the variants named in PMC_VARIANTS.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=${1:-k5}
Z="0,0,0,0,0,0,0,0,0,0"
VARS=${VARS:-"$Z,1 $Z,0,0,4 $Z,0,0,0,4 $Z,0,0,0,6 $Z,0,0,0,8"}
bash tools/ab.sh $TAG $VARS || exit 1
for v in ${PMC_VARIANTS:-}; do
  DCN_EXP=$v bash tools/pmc_pass.sh ${TAG}_$v || exit 1
done
