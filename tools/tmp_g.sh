set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 200 bash tools/sq_passes.sh sq6 "FETCH_SIZE" "WRITE_SIZE" "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_FLAT SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_FLAT SQ_WAIT_INST_ANY" && python tools/pmc_table.py gpurun_out/sq6 k_reduce_edges
