#!/bin/bash
# Quick GPU check: the GPU test suite and one bench line.  Output: gpurun_out/$TAG/
set -o pipefail
TAG=${1:-quick}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 420 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 && echo PYTEST_OK &&
timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > $O/bench.json 2> $O/bench.err && echo BENCH_OK && cat $O/bench.json
