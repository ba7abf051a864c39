#!/bin/bash
# Round 2, first GPU call: the GPU suite (new full-size / ndist tests), one
# bench line, and the first counter passes of the 12-channel long-range
# affinity scan (configs[3]).  Output: gpurun_out/$TAG/
set -o pipefail
TAG=${1:-r2a}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 150 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?; echo "PYTEST rc=$rc"; [ $rc -le 1 ] &&
timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > $O/bench.json 2> $O/bench.err && echo BENCH_OK && cat $O/bench.json &&
CTG_PROF_SIZE=1024 timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/lr_trace -o run -- \
    python tools/prof_scan.py lr > $O/lr_trace.log 2>&1 && echo LR_TRACE_OK &&
CTG_PROF_SIZE=1024 timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/lr_fetch -o run -- \
    python tools/prof_scan.py lr > $O/lr_fetch.log 2>&1 && echo LR_FETCH_OK &&
CTG_PROF_SIZE=1024 timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/lr_write -o run -- \
    python tools/prof_scan.py lr > $O/lr_write.log 2>&1 && echo LR_WRITE_OK
