#!/bin/bash
# GPU test suite only (optionally a -k filter), then the default bench line.
set -o pipefail
TAG=${1:-tests}
K=${2:-}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$TAG
mkdir -p $O
if [ -n "$K" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread -k "$K" > $O/pytest_gpu.log 2>&1
else
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > $O/pytest_gpu.log 2>&1
fi
rc=$?; echo "PYTEST rc=$rc"; tail -3 $O/pytest_gpu.log; grep -E "FAILED|Error" $O/pytest_gpu.log | head -20; [ $rc -eq 0 ] || exit 1
timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > $O/bench.json 2> $O/bench.err || exit 1
python -c "import json; d=json.load(open('$O/bench.json')); print('BENCH', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['frac'], d['phase_ms'])"
