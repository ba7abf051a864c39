#!/bin/bash
# long-range affinity filter: parity, then Bloom vs exact set A/B
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/lrb; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py tests/test_gpu_blocks.py tests/test_gpu_fullsize.py::test_configs3_long_range_affinities_edge_filter \
  -k "aff or long or lr or Aff" > $O/pytest.log 2>&1; rc=$?; tail -5 $O/pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python tools/ab_variants.py lr512,lr1024,nn1024 base base@CTG_LR_FILTER=exact > $O/ab.jsonl 2> $O/ab.err; rc=$?
cat $O/ab.jsonl; exit $rc
