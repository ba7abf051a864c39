set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 200 python tools/ablate2.py v5c@0@4 v5c@0@8 v5c@64@4 v5c@128@4 v5c@32@4 2>&1 | grep -v amdgpu.ids
export CTG_CHECK_PLANES=4
timeout -k 10 200 bash tools/sq_passes.sh sq5 && python tools/pmc_table.py gpurun_out/sq5
