#!/bin/bash
# Round-3 iteration: GPU suite, affinity grouped-fold A/B, occupancy probe,
# N=2 gloo rehearsal.  usage: tools/r3_iter.sh TAG
set -o pipefail
TAG=${1:-r3iter}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
tail -1 $O/pytest_gpu.log; grep FAILED $O/pytest_gpu.log | head -5; [ $rc -eq 0 ] || exit 1
timeout -k 10 500 python tools/ab_variants.py lr1024,nn1024 base noaffgroup base > $O/ab_aff.jsonl 2> $O/ab_aff.err || exit 1
cat $O/ab_aff.jsonl
timeout -k 10 300 python tools/ab_variants.py b512 base base@CTG_SCAN_LDS_PAD=2048 > $O/ab_occ.jsonl 2> $O/ab_occ.err || exit 1
cat $O/ab_occ.jsonl
bash tools/rehearse_n2.sh $TAG > /dev/null || exit 1
grep '^{' $O/bench_n2.json | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("N2", d["ms_per_step"], d["value"], d["exchange_host_reads_per_step"], d["phase_ms"])'
