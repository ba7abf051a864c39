#!/bin/bash
# Bench lines under several environment sets: tools/gpu_ab_sets.sh TAG "configs" "A=1,B=2" "A=3" ...
# (each set is a comma-separated list of VAR=value; "-" = the default environment)
set -o pipefail
TAG=$1; CFGS=$2; shift 2
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$TAG
mkdir -p $O
i=0
for set in "$@"; do
  envs=(); [ "$set" != "-" ] && IFS=',' read -ra envs <<< "$set"
  for c in $CFGS; do
    env "${envs[@]}" timeout -k 10 300 python bench.py --config $c --steps 10 --warmup 2 --no-cpu-baseline > $O/bench_c${c}_$i.json 2> $O/bench_c${c}_$i.err || { echo "CONFIG $c [$set] FAILED"; tail -5 $O/bench_c${c}_$i.err; exit 1; }
    echo "C$c [$set] $(python -c "import json; d=json.load(open('$O/bench_c${c}_$i.json')); print(d['value'], d['ms_per_step'], d.get('phase_ms'))")"
  done
  i=$((i+1))
done
