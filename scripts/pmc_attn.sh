#!/bin/bash
# SQ counters of the C5 forward's kernels (scripts/prof_kernels.py --what c5fwd) under a given
# option setting; two --pmc passes, each under its own limit.
#   scripts/pmc_attn.sh TAG emb_proj=0
set -u
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/$1
OPT=$2
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
i=0
for c in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE" \
         "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_VMEM SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAVES SQ_ACTIVE_INST_SCA GRBM_COUNT" \
         "TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d "$OUT/pmc$i" -o run -- python3 "$ROOT/scripts/prof_kernels.py" --what c5fwd --calls 3 --opt "$OPT" > "$OUT/pmc$i.log" 2>&1
  rc=$?
  echo "pass $i rc=$rc"
  if [ $rc -ne 0 ]; then exit $rc; fi
done
