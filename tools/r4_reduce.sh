#!/bin/bash
# LDS-staged reduce (k_reduce_edges_lds): GPU parity of the paths that reduce
# narrow records, then the A/B against the one-thread-per-edge loads.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r4r}
mkdir -p $O
unset CTG_LIB
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -1 $O/pytest.log; grep FAILED $O/pytest.log | head; [ $rc -eq 0 ] || exit 1
timeout -k 10 700 python tools/ab_variants.py b2048,b1024c5,b512,lr1024 base base@CTG_REDUCE_LDS=0 > $O/ab.jsonl \
  2> $O/ab.err || { tail -5 $O/ab.err; exit 1; }
cat $O/ab.jsonl
echo R4_REDUCE_DONE
