#!/bin/bash
set -o pipefail
TAG=${1:-r2e}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_workflow.py tests/test_gpu_blocks.py -v -s --timeout 400 --timeout-method thread > $O/pytest_wf.log 2>&1; rc=$?; echo "WF rc=$rc"; tail -3 $O/pytest_wf.log; [ $rc -le 1 ] &&
timeout -k 10 400 python bench.py --config 0 --steps 2 --warmup 1 > $O/bench_c0.json 2> $O/bench_c0.err && echo BENCH0_OK && cat $O/bench_c0.json &&
timeout -k 10 900 python tools/ab_variants.py b512,lr1024,b1024c5 base base@CTG_ABLATE=256 wg1024 > $O/ab.jsonl 2> $O/ab.err && echo AB_OK; grep stamps $O/ab.err
