#!/bin/bash
# One GPU-box evidence run, step by step; stops at the first failure (each step under its own
# time limit). Usage: tools/gpu.sh TAG STEP [STEP ...]
#   test      pytest -m gpu (whole suite), summary in gpurun_out/TAG_pytest_gpu.log
#   testk=EXPR  pytest -m gpu -k EXPR
#   smoke     __graft_entry__.smoke()
#   bench     the default bench line (config 3 + config-4/2/5 legs, CPU baselines)
#   prof3 / prof4 / prof5 / prof2   rocprofv3 kernel stats of a short bench run of that config
#   strong    rocprofv3 kernel stats of config 3 at B = 512 (the strong-scaling shard at N = 1)
#   pmc3 / pmc4 / pmc5   FETCH_SIZE and WRITE_SIZE passes (tools/pmc_pass.sh) for that config
#   sq4 / sq3  SQ counters (tools/pmc_sq.sh) for that config
#   mfma2 / mfma3 / mfma4 / mfma5  MFMA-busy counters (tools/pmc_mfma.sh + tools/mfma_summary.py)
#   diag      tools/launch_diag.py (200 config-4 steps per schedule, 40 of config 3, bitwise)
# Env: BENCH_EXTRA (extra bench.py flags for the prof / pmc steps).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
T=$1
shift
Q="--steps 5 --warmup 2 --no-cpu-baseline --no-strong --no-host-path --no-config4 --no-extra-configs --alt-math 0 ${BENCH_EXTRA}"
prof() {  # prof TAG ARGS...
  local tag=$1
  shift
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_$tag -o run --output-format csv -- python3 bench.py "$@" > gpurun_out/${T}_$tag.log 2>&1 || { tail -5 gpurun_out/${T}_$tag.log; return 1; }
  python3 tools/kstats.py gpurun_out/${T}_$tag --top=30
}
for S in "$@"; do
  echo "== $S"
  case $S in
    test)
      timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 120 --timeout-method thread > gpurun_out/${T}_pytest_gpu.log 2>&1 || { tail -30 gpurun_out/${T}_pytest_gpu.log; exit 1; }
      tail -2 gpurun_out/${T}_pytest_gpu.log ;;
    testk=*)
      timeout -k 10 600 python -u -m pytest tests -m gpu -v -rf --timeout 120 --timeout-method thread -k "${S#testk=}" > gpurun_out/${T}_pytest_k.log 2>&1 || { tail -40 gpurun_out/${T}_pytest_k.log; exit 1; }
      tail -3 gpurun_out/${T}_pytest_k.log ;;
    smoke)
      timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" || exit 1 ;;
    bench)
      timeout -k 10 600 python bench.py > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || { tail -20 gpurun_out/${T}_bench.err; exit 1; }
      cut -c1-1200 gpurun_out/${T}_bench.json ;;
    prof3) prof prof3 $Q || exit 1 ;;
    prof4) prof prof4 $Q --config 4 || exit 1 ;;
    prof5) prof prof5 $Q --config 5 || exit 1 ;;
    prof2) prof prof2 $Q --config 2 || exit 1 ;;
    strong) prof strong $Q --global-batch 512 --steps 3 --warmup 1 || exit 1 ;;
    pmc3) bash tools/pmc_pass.sh ${T}c3 || exit 1 ;;
    pmc4) BENCH_ARGS="--config 4 ${BENCH_EXTRA}" bash tools/pmc_pass.sh ${T}c4 || exit 1 ;;
    pmc5) BENCH_ARGS="--config 5 ${BENCH_EXTRA}" bash tools/pmc_pass.sh ${T}c5 || exit 1 ;;
    sq3) bash tools/pmc_sq.sh ${T}c3 || exit 1 ;;
    sq4) BENCH_ARGS="--config 4 ${BENCH_EXTRA}" bash tools/pmc_sq.sh ${T}c4 || exit 1 ;;
    mfma2|mfma3|mfma4|mfma5)
      c=${S#mfma}
      bash tools/pmc_mfma.sh ${T}c$c --config $c ${BENCH_EXTRA} || { tail -5 gpurun_out/mfma_${T}c$c.log; exit 1; }
      python3 tools/mfma_summary.py gpurun_out/mfma_${T}c$c gpurun_out/${T}_mfma_busy_config$c.json --config=$c || exit 1 ;;
    diag)
      timeout -k 10 300 python -u tools/launch_diag.py --reps 200 --reps3 40 --out gpurun_out/${T}_launch_diag.json > gpurun_out/${T}_launch_diag.log 2>&1 || { tail -3 gpurun_out/${T}_launch_diag.log | cut -c1-600; exit 1; }
      echo "launch_diag ok" ;;
    *) echo "unknown step $S"; exit 2 ;;
  esac
done
echo "gpu.sh $T done"
