#!/bin/bash
# Where the 12-channel long-range scan's HBM reads come from: FETCH_SIZE of
# the face scan for channel subsets, with and without the Bloom probes
# (CTG_ABLATE=512 on the CTG_DIAG build), plus the subset timings.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r4lr}
mkdir -p $O
export CTG_LIB=$PWD/variants/libctg_diag.so CTG_PROF_SIZE=1024 CTG_PROF_CELL=10 CTG_PROF_ITERS=2
run() {  # run <name> <ablate> <channels>
  CTG_ABLATE=$2 CTG_PROF_CHANNELS=$3 timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv \
      -d $O/f_$1 -o run -- python tools/prof_scan.py lr > $O/f_$1.log 2>&1 || return 1
  echo "$1 $(python tools/pmc_table.py $O/f_$1 | tr -s ' ' | tr '\n' ' ')"
}
run all 0 0,1,2,3,4,5,6,7,8,9,10,11 &&
run nn 0 0,1,2 && run nnz 0 0,1,2,3,6,9 && run nny 0 0,1,2,4,7,10 && run nnx 0 0,1,2,5,8,11 &&
run nny_nobloom 512 0,1,2,4,7,10 && run nnx_nobloom 512 0,1,2,5,8,11 && run nnz_nobloom 512 0,1,2,3,6,9 || exit 1
echo R4_LR_DONE
