#!/bin/bash
# PMC passes over tools/prof_scan.py (one counter group per rocprofv3 run; no
# tracing domains combined with --pmc).  Output: gpurun_out/pmc/<pass>/...
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/pmc
mkdir -p $OUT
i=0
for group in "$@"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc $group --output-format csv -d $OUT/p$i -o run -- python tools/prof_scan.py boundary > $OUT/p$i.log 2>&1
  echo "pass $i ok: $group"
done
