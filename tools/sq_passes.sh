#!/bin/bash
# SQ / GRBM counter passes over tools/prof_scan.py (each group its own run).
set -o pipefail
TAG=${1:-sq}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$TAG
mkdir -p $O
i=0
shift
for group in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS GRBM_GUI_ACTIVE" \
             "SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_BRANCH SQ_INSTS_SMEM" "$@"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $group --output-format csv -d $O/p$i -o run -- python tools/prof_scan.py boundary > $O/p$i.log 2>&1 || { echo "pass $i FAILED: $group"; exit 1; }
  echo "pass $i ok: $group"
done
