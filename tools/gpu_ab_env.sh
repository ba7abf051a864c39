#!/bin/bash
# A/B of one environment switch on bench lines: tools/r5_ab.sh TAG VAR "configs" (runs VAR=0 then VAR=1)
set -o pipefail
TAG=${1:-ab}; VAR=$2; CFGS=${3:-"4"}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$TAG
mkdir -p $O
for c in $CFGS; do for v in 0 1; do
  env $VAR=$v timeout -k 10 300 python bench.py --config $c --steps 10 --warmup 2 --no-cpu-baseline > $O/bench_c${c}_$v.json 2> $O/bench_c${c}_$v.err || { echo "CONFIG $c $VAR=$v FAILED"; tail -5 $O/bench_c${c}_$v.err; exit 1; }
  echo "C$c $VAR=$v $(python -c "import json; d=json.load(open('$O/bench_c${c}_$v.json')); print(d['value'], d['ms_per_step'], d.get('phase_ms'))")"
done; done
