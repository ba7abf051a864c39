#!/bin/bash
# GPU suite, then two bench lines and one rocprofv3 kernel-stats pass of the bench.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-qab}
mkdir -p $O
timeout -k 10 420 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 && echo PYTEST_OK &&
timeout -k 10 200 python bench.py --steps 50 --warmup 5 --no-cpu-baseline > $O/bench1.json 2> $O/bench1.err && echo B1_OK &&
timeout -k 10 200 python bench.py --steps 50 --warmup 5 --no-cpu-baseline > $O/bench2.json 2> $O/bench2.err && echo B2_OK &&
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- \
    python bench.py --steps 20 --warmup 3 --no-cpu-baseline > $O/bench_traced.json 2> $O/trace.err && echo TRACE_OK
