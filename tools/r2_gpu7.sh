#!/bin/bash
set -o pipefail
TAG=${1:-r2g}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$TAG
mkdir -p $O
H='tests/test_gpu_blocks.py::test_blocks_independent_of_workspace_history'
CTG_LIB=$PWD/variants/libctg_old.so timeout -k 10 200 python -u -m pytest "$H" -q --timeout 120 --timeout-method thread > $O/old.log 2>&1; echo "OLD rc=$? $(tail -1 $O/old.log)"
timeout -k 10 200 python -u -m pytest "$H" -q --timeout 120 --timeout-method thread > $O/new.log 2>&1; rc=$?; echo "NEW rc=$rc $(tail -1 $O/new.log)"; [ $rc -le 1 ] &&
timeout -k 10 900 python tools/ab_variants.py b512,b1024c5,b2048 base nobulk > $O/ab.jsonl 2> $O/ab.err && echo AB_OK && cat $O/ab.jsonl
