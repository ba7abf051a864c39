#!/bin/bash
# Parity of the face-form affinity tests, then configs[4] build variants
# (narrow fold batch, table fill threshold) and their effect on 2048^3.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r4cv}
mkdir -p $O
unset CTG_LIB
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread \
  > $O/pytest.log 2>&1; rc=$?
tail -1 $O/pytest.log; grep FAILED $O/pytest.log | head; [ $rc -eq 0 ] || exit 1
timeout -k 10 700 python tools/ab_variants.py b1024c5,b2048 base npn2 fill384 fill448 > $O/ab.jsonl 2> $O/ab.err \
  || { tail -5 $O/ab.err; exit 1; }
cat $O/ab.jsonl
echo R4_CV_DONE
