#!/bin/bash
# Face-scan ablation at configs[2] (2048^3, cell 16) and configs[1] (512^3)
# with the diagnostic build (variants/libctg_diag.so: make variant NAME=diag
# EXTRA=-DCTG_DIAG), plus tile knobs of the product build at 2048^3.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r4abl}
mkdir -p $O
CTG_PROF_SIZE=2048 CTG_PROF_CELL=16 timeout -k 10 400 python tools/ablate2.py diag@0 diag@8 diag@32 diag@64 diag@128 diag@256 \
  > $O/ablate_2048.jsonl 2> $O/ablate_2048.err || { tail -5 $O/ablate_2048.err; exit 1; }
cat $O/ablate_2048.jsonl; grep stamps $O/ablate_2048.err
CTG_PROF_SIZE=512 CTG_PROF_CELL=10 timeout -k 10 200 python tools/ablate2.py diag@0 diag@8 diag@32 diag@64 diag@128 diag@256 \
  > $O/ablate_512.jsonl 2> $O/ablate_512.err || { tail -5 $O/ablate_512.err; exit 1; }
cat $O/ablate_512.jsonl; grep stamps $O/ablate_512.err
timeout -k 10 400 python tools/ab_variants.py b2048 base base@CTG_TILE_Z=32 base@CTG_TILE_Z=128 base@CTG_XCD_REMAP=0 \
  > $O/knobs_2048.jsonl 2> $O/knobs_2048.err || { tail -5 $O/knobs_2048.err; exit 1; }
cat $O/knobs_2048.jsonl
echo ABLATE_DONE
