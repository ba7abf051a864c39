#!/bin/bash
# Non-temporal affinity sample loads (CTG_NT_AFF, variants/libctg_ntoff.so =
# ordinary loads) + the capped narrow-tile depth: parity, A/B, FETCH_SIZE.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r4nt}
mkdir -p $O
unset CTG_LIB
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -x -v --timeout 500 \
  --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -1 $O/pytest.log; grep FAILED $O/pytest.log | head; [ $rc -eq 0 ] || exit 1
timeout -k 10 600 python tools/ab_variants.py lr1024,nn1024,b2048 base ntoff > $O/ab.jsonl 2> $O/ab.err \
  || { tail -5 $O/ab.err; exit 1; }
cat $O/ab.jsonl
export CTG_PROF_SIZE=1024 CTG_PROF_CELL=10 CTG_PROF_ITERS=2
for v in base ntoff; do
  if [ $v = ntoff ]; then export CTG_LIB=$PWD/variants/libctg_ntoff.so; fi
  timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/f_$v -o run -- python tools/prof_scan.py lr \
    > $O/f_$v.log 2>&1 || exit 1
  echo "$v $(python tools/pmc_table.py $O/f_$v | tr -s ' ' | tr '\n' ' ')"
done
echo R4_NT_DONE
