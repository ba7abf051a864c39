#!/bin/bash
# SQ counter passes of the face scan (512^3, tools/prof_scan.py) under each
# CTG_ABLATE value given: one rocprofv3 --pmc run per (ablate, group).
set -o pipefail
TAG=${1:-sqa}
shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$TAG
mkdir -p $O
for ab in "$@"; do
  i=0
  for group in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS GRBM_GUI_ACTIVE" \
               "SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_BRANCH SQ_INSTS_SMEM"; do
    i=$((i+1))
    CTG_ABLATE=$ab timeout -s KILL 90 rocprofv3 --pmc $group --output-format csv -d $O/a${ab}_p$i -o run -- python tools/prof_scan.py boundary > $O/a${ab}_p$i.log 2>&1 || { echo "pass $ab/$i FAILED"; exit 1; }
  done
  echo "== ablate $ab"; python tools/pmc_table.py $O/a${ab}_p1 ; python tools/pmc_table.py $O/a${ab}_p2
done
