#!/bin/bash
# Full GPU suite, smoke, default bench line and every BASELINE config line.
set -o pipefail
TAG=${1:-full}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 400 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?; echo "PYTEST rc=$rc"; tail -2 $O/pytest_gpu.log; grep FAILED $O/pytest_gpu.log | head; [ $rc -le 1 ] &&
timeout -k 10 200 python -c 'import __graft_entry__ as g; g.smoke()' > $O/smoke.log 2>&1 && echo SMOKE_OK &&
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err && echo BENCH_OK && cat $O/bench.json &&
for c in 1 4 3 3lr 0; do
  if [ "$c" = 0 ]; then CB="--steps 3"; else CB="--steps 5 --no-cpu-baseline"; fi
  timeout -k 10 500 python bench.py --config $c --warmup 1 $CB > $O/bench_c$c.json 2> $O/bench_c$c.err || { echo "CONFIG $c FAILED"; exit 1; }
  echo "CONFIG_${c}_OK $(python -c "import json; d=json.load(open('$O/bench_c$c.json')); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d.get('phase_ms') or d.get('stage_s'))")"
done
