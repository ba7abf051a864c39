#!/bin/bash
# bench.py --config lines under env settings: ab_cfg.sh TAG "ENV=.. ENV=..@config" ...
set -o pipefail
TAG=${1:-abc}; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$TAG
mkdir -p $O
i=0
for spec in "$@"; do
  i=$((i+1)); envs=${spec%@*}; cfg=${spec##*@}
  env $envs timeout -k 10 300 python bench.py --config $cfg --steps 5 --warmup 1 --no-cpu-baseline > $O/c$i.json 2> $O/c$i.err || { echo "FAILED $spec"; exit 1; }
  python -c "import json,sys; d=json.load(open('$O/c$i.json')); print('$spec', d['ms_per_step'], d['phase_ms'])"
done
