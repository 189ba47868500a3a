#!/bin/bash
# SQ / GRBM counters of the C5 forward and C2 encode kernels: one --pmc pass per counter group, each
# under its own time limit (the box refuses combined trace domains), over scripts/prof_kernels.py.
# Raw rocprofv3 output stays in /tmp on the box (it exceeds what gpurun copies back); per-kernel
# means go to gpurun_out/TAG/p<i>.txt (scripts/pmc_db.py).
# Usage: scripts/pmc_sas.sh TAG [WHAT] [--match NAME]   (WHAT: c5fwd,c2 by default)
set -u
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/$1
WHAT=${2:-c5fwd,c2}
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
i=0
for c in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS" \
         "SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE GRBM_COUNT" \
         "SQ_INSTS_SALU SQ_INSTS_VMEM SQ_INSTS_SMEM SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM SQ_WAVES SQ_ACTIVE_INST_SCA SQ_INSTS_BRANCH"; do
  i=$((i+1))
  rm -rf /tmp/gr_pmc_p$i
  timeout -s KILL 90 rocprofv3 --pmc $c -d /tmp/gr_pmc_p$i -o p$i -- python3 "$ROOT/scripts/prof_kernels.py" --what "$WHAT" > "$OUT/p$i.log" 2>&1
  rc=$?
  echo "pass $i rc=$rc"
  if [ $rc -ne 0 ]; then exit $rc; fi
  python3 "$ROOT/scripts/pmc_db.py" $(find /tmp/gr_pmc_p$i -name '*.db') > "$OUT/p$i.txt" 2>&1 || \
    find /tmp/gr_pmc_p$i -type f | head -20 >> "$OUT/p$i.txt"
done
