#!/bin/bash
# GPU suite (batched-blocks tests first) and the default bench line.
set -o pipefail
TAG=${1:-r2b}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_blocks.py -v --timeout 120 --timeout-method thread > $O/pytest_blocks.log 2>&1; rc=$?; echo "BLOCKS rc=$rc"; tail -3 $O/pytest_blocks.log; [ $rc -le 1 ] &&
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread --deselect tests/test_gpu_blocks.py > $O/pytest_gpu.log 2>&1; rc=$?; echo "PYTEST rc=$rc"; tail -3 $O/pytest_gpu.log; [ $rc -le 1 ] &&
timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > $O/bench.json 2> $O/bench.err && echo BENCH_OK && cat $O/bench.json
