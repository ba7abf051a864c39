#!/bin/bash
# One GPU call for a round's evidence: GPU test suite, the bench line, the
# rocprofv3 kernel-trace stats of the same bench command, FETCH_SIZE /
# WRITE_SIZE passes of the face scan (each its own rocprofv3 run), and the
# extra BASELINE config lines.  Output: gpurun_out/$TAG/...
set -o pipefail
TAG=${1:-r1}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 420 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 && echo PYTEST_OK &&
timeout -k 10 200 python bench.py --steps 20 --warmup 3 > $O/bench.json 2> $O/bench.err && echo BENCH_OK &&
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- \
    python bench.py --steps 20 --warmup 3 --no-cpu-baseline > $O/bench_traced.json 2> $O/trace.err && echo TRACE_OK &&
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -o run -- \
    python tools/prof_scan.py boundary > $O/pmc_fetch.log 2>&1 && echo FETCH_OK &&
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write -o run -- \
    python tools/prof_scan.py boundary > $O/pmc_write.log 2>&1 && echo WRITE_OK &&
for c in 4 3 3lr 2; do
  timeout -k 10 300 python bench.py --config $c --steps 5 --warmup 1 --no-cpu-baseline > $O/bench_c$c.json 2> $O/bench_c$c.err || { echo "CONFIG $c FAILED"; exit 1; }
  echo "CONFIG_${c}_OK"
done
