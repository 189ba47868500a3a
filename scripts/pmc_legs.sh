#!/bin/bash
# HBM traffic per bench leg (MI355X_MICROARCH.md §HBM): rocprofv3 --pmc FETCH_SIZE and --pmc
# WRITE_SIZE in separate passes over `bench.py --legs LEG`, raw output in /tmp on the box, summarised
# by scripts/pmc_traffic.py into gpurun_out/TAG/traffic.json (copy to profiles/traffic.json).
# Usage: scripts/pmc_legs.sh TAG [legs...]   (default: c2 sasrec c5 shard train)
set -u
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
TAG=$1; shift
LEGS=${*:-c2 sasrec c5 shard train}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
specs=""
for leg in $LEGS; do
  for c in FETCH_SIZE WRITE_SIZE; do
    rm -rf /tmp/gr_pmc_${leg}_$c
    timeout -k 10 240 rocprofv3 --pmc $c --output-format csv -d /tmp/gr_pmc_${leg}_$c -o run -- \
      python3 "$ROOT/bench.py" --legs $leg --steps 3 --warmup 1 --no-cpu-baseline --spinup-s 0 \
      > "$OUT/pmc_${leg}_$c.log" 2>&1
    rc=$?
    echo "pmc $leg $c rc=$rc"
    if [ $rc -ne 0 ]; then exit $rc; fi
  done
  specs="$specs $leg=/tmp/gr_pmc_${leg}_FETCH_SIZE,/tmp/gr_pmc_${leg}_WRITE_SIZE"
done
python3 "$ROOT/scripts/pmc_traffic.py" --tag "$TAG" $specs > "$OUT/traffic.json"
