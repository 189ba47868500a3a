#!/bin/bash
# One GPU-box session: GPU tests, smoke, bench, rocprofv3 kernel stats.  Every GPU step has its own
# time limit; a fault / abort / timeout (exit codes other than 0 and 1) ends the script at once.
# Usage: scripts/gpu_check.sh [tag] [steps...]   steps: tests smoke bench prof pmc (default: all but pmc)
set -u
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
TAG=${1:-run}; shift || true
STEPS=${*:-tests smoke bench prof}
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
  tail -n 30 "$OUT/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "!! $name ended with $rc: stopping"; exit $rc; fi
  return 0
}

for s in $STEPS; do
  case $s in
    tests) step pytest_gpu 1200 python -m pytest tests -m gpu -q -rs ;;
    smoke) step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) step bench 900 python bench.py ;;
    trace_rq)
      export TMPDIR=/tmp
      cd /tmp
      step trace_rq 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace_rq" -o run -- python3 "$ROOT/scripts/prof_rq.py" --fused 1 && \
      step trace_rq4 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace_rq4" -o run -- python3 "$ROOT/scripts/prof_rq.py" --fused 1 --L 4 --K 1024
      cd "$ROOT" ;;
    ab) step ab_rq 600 python scripts/ab_rq.py && step ab_rq_4x1024 600 python scripts/ab_rq.py --L 4 --K 1024 ;;
    prof)
      export TMPDIR=/tmp
      cd /tmp
      step rocprof 900 rocprofv3 --kernel-trace --stats --output-format csv \
          -d /tmp/gr_rocprof -o run -- python3 "$ROOT/bench.py" --steps 10 --warmup 3 --no-cpu-baseline
      # the full trace is tens of MB (gpurun copies back <= 64 MiB): keep the stats and a per-launch-shape summary
      mkdir -p "$OUT/rocprof"
      cp /tmp/gr_rocprof/run_kernel_stats.csv "$OUT/rocprof/" 2>/dev/null
      python3 "$ROOT/scripts/trace_stats.py" /tmp/gr_rocprof/run_kernel_trace.csv --top 60 > "$OUT/rocprof/trace_stats.csv" 2>&1
      cd "$ROOT" ;;
    micro)
      step micro_valu 300 python scripts/micro/mfma_valu.py ;;
    pmc)  # HBM traffic: FETCH_SIZE and WRITE_SIZE in separate passes (MI355X_MICROARCH.md §HBM)
      export TMPDIR=/tmp
      for c in FETCH_SIZE WRITE_SIZE; do
        cd /tmp
        step pmc_$c 900 rocprofv3 --pmc $c --output-format csv \
            -d "$OUT/pmc_$c" -o run -- python3 "$ROOT/bench.py" --steps 5 --warmup 2 --no-cpu-baseline
        cd "$ROOT"
      done ;;
    pmc3)  # HBM bytes per kernel and bench leg (FETCH_SIZE / WRITE_SIZE, separate passes): scripts/pmc_legs.sh
      step pmc_legs 1100 bash "$ROOT/scripts/pmc_legs.sh" "$TAG" ;;
    pmc2)  # HBM bytes per kernel (FETCH_SIZE / WRITE_SIZE in separate passes) + SQ counters, RQ and SASRec
      export TMPDIR=/tmp
      cd /tmp
      for c in FETCH_SIZE WRITE_SIZE "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES" "GRBM_GUI_ACTIVE SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM"; do
        tag=$(echo $c | cut -d' ' -f1)
        step pmc_rq_$tag 120 rocprofv3 --pmc $c --output-format csv -d "$OUT/pmc_rq_$tag" -o run -- python3 "$ROOT/scripts/prof_rq.py" --iters 5 && \
        step pmc_sas_$tag 120 rocprofv3 --pmc $c --output-format csv -d "$OUT/pmc_sas_$tag" -o run -- python3 "$ROOT/scripts/prof_sas.py" --iters 5
      done
      cd "$ROOT" ;;
    pmcrq)  # SQ counters of the RQ encode kernels (one variant per pass)
      export TMPDIR=/tmp
      cd /tmp
      rocprofv3 -L > "$OUT/counters_list.txt" 2>&1 || true
      for f in 1 0; do
        step pmcrq_f$f 600 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES \
            --output-format csv -d "$OUT/pmcrq_f$f" -o run -- python3 "$ROOT/scripts/prof_rq.py" --fused $f
        step pmcrq2_f$f 600 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE TA_BUSY_avr \
            --output-format csv -d "$OUT/pmcrq2_f$f" -o run -- python3 "$ROOT/scripts/prof_rq.py" --fused $f
      done
      cd "$ROOT" ;;
  esac
done
echo "== done"
