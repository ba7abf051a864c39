#!/bin/bash
# Fold-phase ablations of the diagnostic build at configs[2] (2048^3) and the
# s_memtime split incl. the prefetch wait (ablate 256).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r4abl2}
mkdir -p $O
CTG_PROF_SIZE=2048 CTG_PROF_CELL=16 timeout -k 10 500 python tools/ablate2.py diag@0 diag@256 diag@32 diag@64 diag@128 diag@1024 diag@2048 diag@3200 \
  > $O/ablate_2048.jsonl 2> $O/ablate_2048.err || { tail -5 $O/ablate_2048.err; exit 1; }
cat $O/ablate_2048.jsonl; grep stamps $O/ablate_2048.err | head -3
CTG_PROF_SIZE=512 CTG_PROF_CELL=10 timeout -k 10 200 python tools/ablate2.py diag@0 diag@256 diag@64 diag@1024 \
  > $O/ablate_512.jsonl 2> $O/ablate_512.err || { tail -5 $O/ablate_512.err; exit 1; }
cat $O/ablate_512.jsonl; grep stamps $O/ablate_512.err | head -3
echo ABLATE2_DONE
