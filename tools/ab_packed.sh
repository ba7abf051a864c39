#!/bin/bash
# A/B of the packed key+slot record sort (CTG_SORT_PACKED) plus the GPU suite.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-abpk}
mkdir -p $O
timeout -k 10 420 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 && echo PYTEST_OK &&
CTG_SORT_PACKED=0 timeout -k 10 200 python bench.py --steps 50 --warmup 5 --no-cpu-baseline > $O/bench_off.json 2> $O/bench_off.err && echo OFF_OK &&
timeout -k 10 200 python bench.py --steps 50 --warmup 5 --no-cpu-baseline > $O/bench_on.json 2> $O/bench_on.err && echo ON_OK &&
CTG_SORT_PACKED=0 timeout -k 10 200 python bench.py --steps 50 --warmup 5 --no-cpu-baseline > $O/bench_off2.json 2> $O/bench_off2.err && echo OFF2_OK &&
timeout -k 10 200 python bench.py --steps 50 --warmup 5 --no-cpu-baseline > $O/bench_on2.json 2> $O/bench_on2.err && echo ON2_OK
