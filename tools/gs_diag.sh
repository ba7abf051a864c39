#!/bin/bash
# Per-phase s_memtime sums of the group sort's k_gs_sort (configs[4] and [2]):
# needs the diagnostic build (make -C cluster_tools_amd/csrc variant NAME=diag EXTRA=-DCTG_DIAG).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/gsd
mkdir -p $O
export CTG_LIB=$GRAFT_REPO_ROOT/variants/libctg_diag.so CTG_GS_DIAG=1
timeout -k 10 200 python bench.py --config 4 --steps 2 --warmup 1 --no-cpu-baseline > $O/b4.json 2> $O/b4.err && grep gs_sort $O/b4.err | tail -2 &&
timeout -k 10 200 python bench.py --config 2 --steps 2 --warmup 1 --no-cpu-baseline > $O/b2.json 2> $O/b2.err && grep gs_sort $O/b2.err | tail -1
