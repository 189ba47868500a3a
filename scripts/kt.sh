#!/bin/bash
# Kernel trace of scripts/prof_kernels.py (rocprofv3 --kernel-trace --stats), summarised per launch
# shape into gpurun_out/TAG/trace_stats.csv (the raw trace stays in /tmp on the box).
# Usage: scripts/kt.sh TAG [prof_kernels.py args...]
set -u
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
TAG=$1; shift
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
rm -rf /tmp/gr_kt_$TAG
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/gr_kt_$TAG -o run -- \
  python3 "$ROOT/scripts/prof_kernels.py" "$@" > "$OUT/kt.log" 2>&1
rc=$?
TR=$(find /tmp/gr_kt_$TAG -name '*kernel_trace.csv' | head -1)
python3 "$ROOT/scripts/trace_stats.py" "$TR" --top 30 > "$OUT/trace_stats.csv" 2>&1
if [ "${KT_RAW:-0}" = 1 ]; then cp "$TR" "$OUT/kernel_trace.csv"; fi   # small runs: keep the timeline
exit $rc
