#!/bin/bash
# GPU suite, the default bench line, then an A/B of env settings on the
# in-tree build.  usage: iter_ab_env.sh TAG WORKLOADS SPEC...  (SPEC: base@ENV=val,...)
set -o pipefail
TAG=$1; shift
WL=$1; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 420 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
tail -1 $O/pytest_gpu.log; grep FAILED $O/pytest_gpu.log | head -5; [ $rc -eq 0 ] || exit 1
timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > $O/bench.json 2> $O/bench.err || exit 1
python -c "import json; d=json.load(open('$O/bench.json')); print('BENCH', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['frac'], d['phase_ms'])"
timeout -k 10 600 python tools/ab_variants.py $WL "$@" > $O/ab.jsonl 2> $O/ab.err || { tail -5 $O/ab.err; exit 1; }
cat $O/ab.jsonl
