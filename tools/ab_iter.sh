#!/bin/bash
# GPU suite + A/B of variants/libctg_<name>.so against the in-tree build.
# usage: ab_iter.sh TAG WORKLOADS VARIANT...   Output: gpurun_out/$TAG/
set -o pipefail
TAG=$1; shift
WL=$1; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 420 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
tail -1 $O/pytest_gpu.log; grep FAILED $O/pytest_gpu.log | head -5; [ $rc -eq 0 ] || exit 1
timeout -k 10 600 python tools/ab_variants.py $WL base "$@" > $O/ab.jsonl 2> $O/ab.err || { tail -5 $O/ab.err; exit 1; }
cat $O/ab.jsonl
