#!/bin/bash
# One GPU call for a round's profile evidence (output: gpurun_out/$TAG/...):
#  * rocprofv3 --kernel-trace --stats of every bench line: the default
#    (configs[2], 2048^3), configs[1], configs[3] (3-channel, 12-channel),
#    configs[4], and the configs[0] batched per-block scan (tools/prof_blocks.py);
#  * FETCH_SIZE and WRITE_SIZE passes (each its own rocprofv3 run, no tracing
#    domain beside --pmc) of the face scan on the same workloads
#    (tools/prof_scan.py, tools/prof_blocks.py);
#  * summaries gpurun_out/$TAG/pmc_summary[_c<cfg>].json stamped with $SHA
#    (tools/pmc_summary.py), ready to copy into profiles/<round>/.
# usage: tools/round_profile.sh <tag> <git sha of the uploaded tree> [configs]
set -o pipefail
TAG=${1:-r3}
SHA=${2:-unknown}
CONFIGS=${3:-"1 3 3lr 4 2 0"}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$TAG
mkdir -p $O
echo "$SHA" > $O/HEAD_SHA
pmc() {   # pmc <name> <program...>: one FETCH_SIZE pass and one WRITE_SIZE pass
  local name=$1; shift
  timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch_$name -o run -- \
      "$@" > $O/pmc_fetch_$name.log 2>&1 &&
  timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write_$name -o run -- \
      "$@" > $O/pmc_write_$name.log 2>&1 &&
  echo "PMC_${name}_OK"
}
for c in $CONFIGS; do
  case $c in
    1)   S=512;  CELL=10; MODE=boundary; ALG=$((512*512*512*12)); SUF="" ;;
    2)   S=2048; CELL=16; MODE=boundary; ALG=$((2048*2048*2048*12)); SUF="_c2" ;;
    3)   S=1024; CELL=10; MODE=nn;       ALG=$((1024*1024*1024*20)); SUF="_c3" ;;
    3lr) S=1024; CELL=10; MODE=lr;       ALG=$((1024*1024*1024*56)); SUF="_c3lr" ;;
    4)   S=1024; CELL=5;  MODE=boundary; ALG=$((1024*1024*1024*12)); SUF="_c4" ;;
    0)   SUF="_c0" ;;
  esac
  if [ "$c" = 0 ]; then
    CTG_PROF_ITERS=3 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_c0 -o run -- \
        python tools/prof_blocks.py > $O/trace_c0.log 2>&1 && echo TRACE_c0_OK || exit 1
    CTG_PROF_ITERS=2 pmc c0 python tools/prof_blocks.py || exit 1
    ALG=$(grep -o 'feature_scan_bytes=[0-9]*' $O/trace_c0.log | head -1 | cut -d= -f2)
  else
    if [ "$c" = 1 ]; then
      timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_c1 -o run -- \
          python bench.py --config 1 --steps 20 --warmup 3 --no-cpu-baseline > $O/bench_traced_c1.json 2> $O/trace_c1.err
    else
      timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_c$c -o run -- \
          python bench.py --config $c --steps 5 --warmup 1 --no-cpu-baseline > $O/bench_traced_c$c.json 2> $O/trace_c$c.err
    fi || { echo "TRACE_c${c} FAILED"; exit 1; }
    echo "TRACE_c${c}_OK $(cat $O/bench_traced_c$c.json)"
    CTG_PROF_SIZE=$S CTG_PROF_CELL=$CELL CTG_PROF_ITERS=2 pmc c$c python tools/prof_scan.py $MODE || exit 1
    grep -h "^done" $O/pmc_write_c$c.log > $O/records_c$c.txt || true
  fi
  python tools/pmc_summary.py $O/trace_c$c $O/pmc_fetch_c$c $O/pmc_write_c$c $O/pmc_summary$SUF.json $ALG "$SHA" ||
      exit 1
done
echo ROUND_PROFILE_DONE
