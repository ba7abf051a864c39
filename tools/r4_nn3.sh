#!/bin/bash
# Nearest-neighbour affinities as a face scan (MODE_AFF_NN): GPU suite, then
# the A/B against the channel loop (CTG_NN3=0) and the configs[3] line.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r4nn}
mkdir -p $O
unset CTG_LIB
timeout -k 10 800 python -u -m pytest tests -m gpu -x -v --timeout 500 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -1 $O/pytest.log; grep FAILED $O/pytest.log | head; [ $rc -eq 0 ] || exit 1
timeout -k 10 600 python tools/ab_variants.py lr1024,lr512,nn1024 base base@CTG_NN3=0 > $O/ab.jsonl 2> $O/ab.err \
  || { tail -5 $O/ab.err; exit 1; }
cat $O/ab.jsonl
timeout -k 10 300 python bench.py --config 3lr --steps 10 --warmup 2 --no-cpu-baseline > $O/bench_c3lr.json 2> $O/bench_c3lr.err \
  || { tail -5 $O/bench_c3lr.err; exit 1; }
cat $O/bench_c3lr.json
echo R4_NN3_DONE
