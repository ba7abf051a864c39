#!/bin/bash
# Full GPU suite (stop at the first failure), then bench lines of the given configs.
#   tools/r5_full.sh TAG "configs"
set -o pipefail
TAG=${1:-full}
CFGS=${2:-"4 2 1"}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "PYTEST rc=$rc"; tail -3 $O/pytest_gpu.log; grep -E "FAILED|Error" $O/pytest_gpu.log | head -20; [ $rc -eq 0 ] || exit 1
[ "$CFGS" = "-" ] && exit 0
for c in $CFGS; do
  timeout -k 10 300 python bench.py --config $c --steps 10 --warmup 2 --no-cpu-baseline > $O/bench_c$c.json 2> $O/bench_c$c.err || { echo "CONFIG $c FAILED"; tail -5 $O/bench_c$c.err; exit 1; }
  echo "C$c $(python -c "import json; d=json.load(open('$O/bench_c$c.json')); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d.get('records'), d.get('phase_ms'))")"
done
