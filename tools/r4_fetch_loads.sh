#!/bin/bash
# Is the configs[2] scan's read excess (1.38x) in the load pattern itself?
# FETCH_SIZE of the diagnostic build with loads only (CTG_ABLATE=8) vs full.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r4fl}
mkdir -p $O
export CTG_LIB=$PWD/variants/libctg_diag.so CTG_PROF_SIZE=2048 CTG_PROF_CELL=16 CTG_PROF_ITERS=2
for ab in 8 0; do
  CTG_ABLATE=$ab timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/f_$ab -o run -- \
    python tools/prof_scan.py boundary > $O/f_$ab.log 2>&1 || exit 1
  echo "ablate=$ab $(python tools/pmc_table.py $O/f_$ab | tr -s ' ' | tr '\n' ' ')"
done
echo R4_FL_DONE
