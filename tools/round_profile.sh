#!/bin/bash
# One GPU call for a round's profile evidence (output: gpurun_out/$TAG/...):
#  * rocprofv3 --kernel-trace --stats of the default bench line (configs[1]),
#    and of the configs[3] (3-channel, 12-channel) and configs[4] lines;
#  * FETCH_SIZE and WRITE_SIZE passes (each its own rocprofv3 run, no tracing
#    domain beside --pmc) of the face scan on the same workloads
#    (tools/prof_scan.py).
# Summaries: python tools/pmc_summary.py <trace> <pmc_fetch> <pmc_write> <out.json> <alg_bytes>
set -o pipefail
TAG=${1:-r2}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$TAG
mkdir -p $O
prof() {   # prof <name> <env...> -- <prof_scan mode>
  local name=$1 mode=$2 size=$3 cell=$4
  CTG_PROF_SIZE=$size CTG_PROF_CELL=$cell CTG_PROF_ITERS=2 timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE \
      --output-format csv -d $O/pmc_fetch_$name -o run -- python tools/prof_scan.py $mode > $O/pmc_fetch_$name.log 2>&1 &&
  CTG_PROF_SIZE=$size CTG_PROF_CELL=$cell CTG_PROF_ITERS=2 timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE \
      --output-format csv -d $O/pmc_write_$name -o run -- python tools/prof_scan.py $mode > $O/pmc_write_$name.log 2>&1 &&
  echo "PMC_${name}_OK"
}
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- \
    python bench.py --steps 20 --warmup 3 --no-cpu-baseline > $O/bench_traced.json 2> $O/trace.err && echo TRACE_OK &&
prof c1 boundary 512 10 &&
for c in 3 3lr 4; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_c$c -o run -- \
      python bench.py --config $c --steps 5 --warmup 1 --no-cpu-baseline > $O/bench_traced_c$c.json 2> $O/trace_c$c.err &&
  echo "TRACE_c${c}_OK" || exit 1
done &&
prof c3 nn 1024 10 && prof c3lr lr 1024 10 && prof c4 boundary 1024 5
