#!/bin/bash
# ab_run.sh TAG WORKLOADS VARIANT... : tools/ab_variants.py on the GPU box.
set -o pipefail
TAG=$1; shift
WL=$1; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 1000 python tools/ab_variants.py $WL "$@" > $O/ab.jsonl 2> $O/ab.err; rc=$?
cat $O/ab.jsonl
exit $rc
