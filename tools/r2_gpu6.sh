#!/bin/bash
set -o pipefail
TAG=${1:-r2f}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_blocks.py tests/test_gpu_ndist.py -v --timeout 300 --timeout-method thread > $O/pytest_blocks.log 2>&1; rc=$?; echo "BLOCKS rc=$rc"; grep -E "PASSED|FAILED" $O/pytest_blocks.log | sed 's/.*:://' | tr '\n' ' '; echo; [ $rc -le 1 ] &&
timeout -k 10 400 python bench.py --config 0 --steps 2 --warmup 1 > $O/bench_c0.json 2> $O/bench_c0.err && echo BENCH0_OK && cat $O/bench_c0.json
