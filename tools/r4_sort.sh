#!/bin/bash
# In-LDS bucket sort: parity (new tests + the full-size configs[2]/[4] tests)
# and the A/B against rocPRIM (CTG_LDS_SORT=0) on the BASELINE workloads.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r4g}
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -x -v --timeout 600 \
  --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -1 $O/pytest.log; grep FAILED $O/pytest.log | head; [ $rc -eq 0 ] || exit 1
timeout -k 10 600 python tools/ab_variants.py b2048,b1024c5,b512 base base@CTG_LDS_SORT=0 > $O/ab.jsonl 2> $O/ab.err \
  || { tail -5 $O/ab.err; exit 1; }
cat $O/ab.jsonl
echo R4_SORT_DONE
