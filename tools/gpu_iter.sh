#!/bin/bash
# Iteration check on the GPU box: GPU test suite, the default bench line, and
# (with SQ=1) the two SQ counter passes of the face scan.  Output: gpurun_out/$TAG/
set -o pipefail
TAG=${1:-iter}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 420 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
tail -1 $O/pytest_gpu.log; grep FAILED $O/pytest_gpu.log | head -5; [ $rc -eq 0 ] || exit 1
timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > $O/bench.json 2> $O/bench.err || exit 1
python -c "import json; d=json.load(open('$O/bench.json')); print('BENCH', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['frac'], d['phase_ms'])"
if [ "${SQ:-0}" = 1 ]; then
  i=0
  for group in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS GRBM_GUI_ACTIVE" \
               "SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_BRANCH SQ_INSTS_SMEM"; do
    i=$((i+1))
    timeout -s KILL 90 rocprofv3 --pmc $group --output-format csv -d $O/sq$i -o run -- python tools/prof_scan.py boundary > $O/sq$i.log 2>&1 || { echo "SQ pass $i FAILED"; exit 1; }
  done
  python tools/pmc_table.py $O > $O/sq_table.txt && cat $O/sq_table.txt
fi
