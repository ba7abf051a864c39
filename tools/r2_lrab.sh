#!/bin/bash
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/lrab; mkdir -p $O
timeout -k 10 700 python tools/ab_variants.py ${WL:-lr1024} ${VARS:-base@CTG_ABLATE=256 base@CTG_ABLATE=32 base@CTG_ABLATE=8 base@CTG_ABLATE=64 base@CTG_ABLATE=128} > $O/ab.jsonl 2> $O/ab.err; rc=$?
cat $O/ab.jsonl; grep stamps $O/ab.err | tail -3; exit $rc
