#!/bin/bash
# Where the reduction's time goes: bench phase times under CTG_REDUCE_ABLATE
# (0 full, 1 no quantile walk, 2 no record loads, 4 no feature stores, 7 none of them).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-rabl}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 && echo PYTEST_OK &&
for a in 0 1 2 4 7 0; do
  CTG_REDUCE_ABLATE=$a timeout -k 10 200 python bench.py --steps 50 --warmup 5 --no-cpu-baseline > $O/bench_a$a.json 2> $O/bench_a$a.err || exit 1
  echo "A${a}_OK"
done
