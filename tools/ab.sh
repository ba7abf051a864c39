#!/bin/bash
# A/B timing of face-scan variants (variants/libctg_<name>.so) + optional icache pass.
set -o pipefail
TAG=${1:-ab}; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 300 python tools/ablate2.py "$@" > $O/ab.jsonl 2> $O/ab.err && echo AB_OK && cat $O/ab.jsonl
