#!/bin/bash
set -o pipefail
TAG=${1:-q}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_fullsize.py tests/test_gpu_parity.py -v --timeout 400 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; echo "PYTEST rc=$rc"; tail -1 $O/pytest.log; grep FAILED $O/pytest.log | head; [ $rc -le 1 ] &&
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 50 > $O/bench.json 2> $O/bench.err && echo BENCH_OK && python -c "import json; d=json.load(open('$O/bench.json')); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['phase_ms'])" &&
timeout -k 10 300 python bench.py --config 4 --steps 5 --warmup 1 --no-cpu-baseline > $O/bench_c4.json 2> $O/bench_c4.err && python -c "import json; d=json.load(open('$O/bench_c4.json')); print(d['value'], d['ms_per_step'], d['phase_ms'])"
