#!/bin/bash
# Batched-block / workflow tests, the whole GPU suite, bench lines (default, configs[0]).
set -o pipefail
TAG=${1:-r2c}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_blocks.py tests/test_gpu_workflow.py -v -s --timeout 400 --timeout-method thread > $O/pytest_wf.log 2>&1; rc=$?; echo "WF rc=$rc"; tail -3 $O/pytest_wf.log; [ $rc -le 1 ] &&
timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > $O/bench.json 2> $O/bench.err && echo BENCH_OK && cat $O/bench.json &&
timeout -k 10 400 python bench.py --config 0 --steps 2 --warmup 1 > $O/bench_c0.json 2> $O/bench_c0.err && echo BENCH0_OK && cat $O/bench_c0.json &&
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?; echo "PYTEST rc=$rc"; tail -3 $O/pytest_gpu.log
