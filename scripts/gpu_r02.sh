#!/bin/bash
# Round-2 GPU session: parity tests (with the audit JSON), smoke, bench, and one rocprofv3
# kernel-trace run PER BENCH LEG (so no kernel name mixes launch shapes across configs), each split
# by launch shape with scripts/trace_stats.py.  Every GPU step has its own time limit; a fault /
# abort / timeout (exit codes other than 0 and 1) ends the script at once.
# Usage: scripts/gpu_r02.sh TAG [steps...]   steps: tests smoke bench legs pmc
set -u
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
TAG=${1:-run}; shift || true
STEPS=${*:-tests smoke bench legs}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0

step() {  # name, timeout, command...
  local name=$1 t=$2; shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"
  tail -n 12 "$OUT/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "!! $name ended with $rc: stopping"; exit $rc; fi
  return 0
}

for s in $STEPS; do
  case $s in
    tests) GR_PARITY_OUT=$OUT/parity_counts.json step pytest_gpu 1500 \
             python -u -m pytest tests -m gpu -v -rs --timeout 400 --timeout-method thread ;;
    quick) GR_PARITY_OUT=$OUT/parity_counts.json step pytest_quick 900 \
             python -u -m pytest tests -m gpu -v -rs --timeout 300 --timeout-method thread -k "${GR_TESTS_K:-not full_size}" ;;
    smoke) step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) step bench 900 python bench.py ;;
    legs)
      export TMPDIR=/tmp
      for leg in ${GR_LEGS:-c2 calls sasrec c4 c5 shard train}; do
        cd /tmp
        step prof_$leg 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_$leg" -o run -- \
            python3 "$ROOT/bench.py" --legs $leg --steps 10 --warmup 3 --no-cpu-baseline --spinup-s 0.5
        cd "$ROOT"
        python3 scripts/trace_stats.py "$OUT/prof_$leg/run_kernel_trace.csv" --leg $leg > "$OUT/trace_$leg.csv" || true
        rm -f "$OUT/prof_$leg/run_kernel_trace.csv"   # raw traces exceed gpurun's 64 MiB copy-back
      done ;;
    pmc)  # HBM traffic per bench leg and kernel: FETCH_SIZE and WRITE_SIZE in separate passes
      export TMPDIR=/tmp
      specs=""
      for leg in ${GR_PMC_LEGS:-c2 sasrec c5 shard train}; do
        cd /tmp
        for c in FETCH_SIZE WRITE_SIZE; do
          step pmc_${leg}_$c 240 rocprofv3 --pmc $c --output-format csv -d "$OUT/pmc_${leg}_$c" -o run -- \
              python3 "$ROOT/bench.py" --legs $leg --steps 3 --warmup 1 --no-cpu-baseline --spinup-s 0.1
        done
        cd "$ROOT"
        specs="$specs $leg=$OUT/pmc_${leg}_FETCH_SIZE,$OUT/pmc_${leg}_WRITE_SIZE"
      done
      python3 scripts/pmc_traffic.py --tag "$TAG" $specs > "$OUT/traffic.json" ;;
  esac
done
echo "== done"
