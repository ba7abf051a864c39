#!/bin/bash
# Partial table flushes (CTG_PARTIAL_FLUSH variants): parity of the most
# aggressive variant, then the A/B on the BASELINE workloads.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r4h}
mkdir -p $O
CTG_LIB=$PWD/variants/libctg_pf2a3.so timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py \
  tests/test_gpu_fullsize.py -x -v --timeout 600 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -1 $O/pytest.log; grep FAILED $O/pytest.log | head; [ $rc -eq 0 ] || exit 1
timeout -k 10 700 python tools/ab_variants.py b1024c5,b512,b2048 base pf1a2 pf1a4 pf2a3 > $O/ab.jsonl 2> $O/ab.err \
  || { tail -5 $O/ab.err; exit 1; }
cat $O/ab.jsonl
echo R4_PARTIAL_DONE
