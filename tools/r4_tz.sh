#!/bin/bash
# GPU suite on the current build, then the narrow-tile depth (configs[4]) and
# the Bloom bits per edge (12-channel long-range) A/B.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r4tz}
mkdir -p $O
unset CTG_LIB
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -1 $O/pytest.log; grep FAILED $O/pytest.log | head; [ $rc -eq 0 ] || exit 1
timeout -k 10 600 python tools/ab_variants.py b1024c5 base@CTG_TILE_Z_NARROW=8 base@CTG_TILE_Z_NARROW=12 base \
  base@CTG_TILE_Z_NARROW=24 base@CTG_TILE_Z_NARROW=32 > $O/ab_c4.jsonl 2> $O/ab_c4.err || { tail -5 $O/ab_c4.err; exit 1; }
cat $O/ab_c4.jsonl
timeout -k 10 600 python tools/ab_variants.py lr1024 base base@CTG_BLOOM_BPK=48 base@CTG_BLOOM_BPK=64 \
  > $O/ab_lr.jsonl 2> $O/ab_lr.err || { tail -5 $O/ab_lr.err; exit 1; }
cat $O/ab_lr.jsonl
echo R4_TZ_DONE
