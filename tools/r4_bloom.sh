#!/bin/bash
# Owner-blocked Bloom filter + lazy shard-size read: GPU tests of the affected
# paths, the 12-channel A/B against the previous filter (variants/libctg_oldbloom.so),
# a FETCH_SIZE pass of the 12-channel scan, the world-1 distributed step, and
# the configs[4] tile-depth A/B.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r4b}
mkdir -p $O
unset CTG_LIB
timeout -k 10 600 python -u -m pytest tests/test_gpu_dist.py tests/test_gpu_parity.py tests/test_gpu_ndist.py \
  tests/test_gpu_blocks.py -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -1 $O/pytest.log; grep FAILED $O/pytest.log | head; [ $rc -eq 0 ] || exit 1
timeout -k 10 600 python tools/ab_variants.py lr1024,lr512 base oldbloom > $O/ab_lr.jsonl 2> $O/ab_lr.err \
  || { tail -5 $O/ab_lr.err; exit 1; }
cat $O/ab_lr.jsonl
CTG_PROF_SIZE=1024 CTG_PROF_CELL=10 CTG_PROF_ITERS=2 timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE \
  --output-format csv -d $O/f_all -o run -- python tools/prof_scan.py lr > $O/f_all.log 2>&1 || exit 1
python tools/pmc_table.py $O/f_all
timeout -k 10 300 python tools/ab_variants.py b1024c5 base base@CTG_TILE_Z=64 base@CTG_TILE_Z=16 > $O/ab_c4.jsonl \
  2> $O/ab_c4.err || { tail -5 $O/ab_c4.err; exit 1; }
cat $O/ab_c4.jsonl
bash tools/r4_distph.sh ${1:-r4b} || exit 1
timeout -k 10 300 python tools/exit_floor.py > $O/exit_floor.jsonl 2> $O/exit_floor.err || { tail -5 $O/exit_floor.err; exit 1; }
cat $O/exit_floor.jsonl
echo R4_BLOOM_DONE
