#!/bin/bash
# Tile depth for the narrow (fragmented) tile and Bloom bits per edge.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r4tz}
mkdir -p $O
unset CTG_LIB
timeout -k 10 600 python tools/ab_variants.py b1024c5 base@CTG_TILE_Z=8 base@CTG_TILE_Z=12 base@CTG_TILE_Z=16 \
  base@CTG_TILE_Z=24 base > $O/ab_c4.jsonl 2> $O/ab_c4.err || { tail -5 $O/ab_c4.err; exit 1; }
cat $O/ab_c4.jsonl
timeout -k 10 600 python tools/ab_variants.py b512,nn1024 base base@CTG_TILE_Z=16 > $O/ab_b512.jsonl 2> $O/ab_b512.err \
  || { tail -5 $O/ab_b512.err; exit 1; }
cat $O/ab_b512.jsonl
timeout -k 10 600 python tools/ab_variants.py lr1024 base base@CTG_BLOOM_BPK=48 base@CTG_BLOOM_BPK=64 \
  > $O/ab_lr.jsonl 2> $O/ab_lr.err || { tail -5 $O/ab_lr.err; exit 1; }
cat $O/ab_lr.jsonl
echo R4_TZ_DONE
