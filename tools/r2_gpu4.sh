#!/bin/bash
# Workflow repeatability / concurrency tests, batched-call trace, two-choice A/B.
set -o pipefail
TAG=${1:-r2d}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_workflow.py tests/test_gpu_blocks.py tests/test_gpu_parity.py -v -s --timeout 400 --timeout-method thread > $O/pytest_wf.log 2>&1; rc=$?; echo "WF rc=$rc"; tail -5 $O/pytest_wf.log; [ $rc -le 1 ] &&
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/blocks_trace -o run -- python tools/prof_blocks.py > $O/blocks.log 2>&1 && echo BLOCKS_TRACE_OK && cat $O/blocks.log &&
timeout -k 10 900 python tools/ab_variants.py b512,lr1024,b1024c5,nn1024 base tc0 > $O/ab.jsonl 2> $O/ab.err && echo AB_OK
