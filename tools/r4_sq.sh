#!/bin/bash
# SQ counters of the configs[2] face scan (one pass, 8 SQ counters, no trace
# domain beside --pmc): where the waves' cycles go.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r4sq}
mkdir -p $O
unset CTG_LIB
CTG_PROF_SIZE=2048 CTG_PROF_CELL=16 CTG_PROF_ITERS=2 timeout -s KILL 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY \
  SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_LDS --output-format csv \
  -d $O/sq1 -o run -- python tools/prof_scan.py boundary > $O/sq1.log 2>&1 || exit 1
python tools/pmc_table.py $O/sq1 > $O/sq1.txt; cat $O/sq1.txt
CTG_PROF_SIZE=2048 CTG_PROF_CELL=16 CTG_PROF_ITERS=2 timeout -s KILL 240 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT \
  SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_BRANCH SQ_WAVES SQ_BUSY_CYCLES SQ_INSTS_SMEM \
  --output-format csv -d $O/sq2 -o run -- python tools/prof_scan.py boundary > $O/sq2.log 2>&1 || exit 1
python tools/pmc_table.py $O/sq2 > $O/sq2.txt; cat $O/sq2.txt
echo R4_SQ_DONE
