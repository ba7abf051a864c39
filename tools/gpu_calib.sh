#!/bin/bash
# Counter calibration (tools/calib.hip): kernel trace + one FETCH_SIZE and one
# WRITE_SIZE pass, each its own rocprofv3 run.
set -o pipefail
TAG=${1:-calib}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$TAG
mkdir -p $O
timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- ./tools/calib 3 > $O/calib.json 2> $O/trace.log &&
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o run -- ./tools/calib 1 > /dev/null 2> $O/fetch.log &&
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write -o run -- ./tools/calib 1 > /dev/null 2> $O/write.log &&
echo CALIB_OK
