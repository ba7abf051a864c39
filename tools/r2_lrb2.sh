#!/bin/bash
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/lrb2; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py tests/test_gpu_blocks.py tests/test_gpu_ndist.py > $O/pytest.log 2>&1; rc=$?; tail -3 $O/pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python tools/ab_variants.py lr1024 base base@CTG_BLOOM_BPK=8 base@CTG_BLOOM_BPK=32 > $O/ab.jsonl 2> $O/ab.err; rc=$?
cat $O/ab.jsonl; exit $rc
