#!/bin/bash
# World-1 distributed step after the device-built shard sizes, and cheap
# environment knobs at configs[4] / configs[2].
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r4k}
mkdir -p $O
unset CTG_LIB
bash tools/r4_distph.sh ${1:-r4k} || exit 1
timeout -k 10 600 python tools/ab_variants.py b1024c5 base base@CTG_XCD_REMAP=0 base@CTG_CHECK_PLANES=4 \
  base@CTG_CHECK_PLANES=16 > $O/ab_c4.jsonl 2> $O/ab_c4.err || { tail -5 $O/ab_c4.err; exit 1; }
cat $O/ab_c4.jsonl
echo R4_KNOBS_DONE
