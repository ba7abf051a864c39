#!/bin/bash
# Which earlier test makes test_blocks_affinity_features fail?  Each pair in a fresh process.
set -o pipefail
TAG=${1:-bis}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$TAG
mkdir -p $O
A='tests/test_gpu_blocks.py::test_blocks_affinity_features'
for T in "tests/test_gpu_workflow.py::test_workflow_affinities_repeatable" "tests/test_gpu_workflow.py::test_workflow_configs0_geometry"; do
  timeout -k 10 200 python -u -m pytest "$T" "$A" -q --timeout 120 --timeout-method thread -p no:randomly > $O/pair.log 2>&1; rc=$?
  echo "$rc :: $T :: $(tail -1 $O/pair.log)"
  [ $rc -le 1 ] || exit $rc
done
