#!/bin/bash
# The extra BASELINE config bench lines only.  Output: gpurun_out/$TAG/bench_c*.json
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-cfg}
mkdir -p $O
for c in 4 3 3lr 2; do
  timeout -k 10 300 python bench.py --config $c --steps 5 --warmup 1 --no-cpu-baseline > $O/bench_c$c.json 2> $O/bench_c$c.err || { echo "CONFIG $c FAILED"; exit 1; }
  echo "CONFIG_${c}_OK"
done
