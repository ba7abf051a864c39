#!/bin/bash
# One GPU call: kernel-trace stats of bench.py, FETCH_SIZE / WRITE_SIZE passes
# (each its own rocprofv3 run, no tracing domains beside --pmc), the
# loads-only ablation pass for the FETCH_SIZE calibration, and the per-phase
# ablation timings.  Output: gpurun_out/$TAG/...
set -o pipefail
TAG=${1:-r1}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- \
    python bench.py --steps 20 --warmup 3 --no-cpu-baseline > $O/bench_traced.json 2> $O/trace.err && echo TRACE_OK &&
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -o run -- \
    python tools/prof_scan.py boundary > $O/pmc_fetch.log 2>&1 && echo FETCH_OK &&
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write -o run -- \
    python tools/prof_scan.py boundary > $O/pmc_write.log 2>&1 && echo WRITE_OK &&
CTG_ABLATE=8 timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch_loads -o run -- \
    python tools/prof_scan.py boundary > $O/pmc_fetch_loads.log 2>&1 && echo FETCH_LOADS_OK &&
timeout -k 10 240 python tools/ablate2.py > $O/ablate.jsonl 2> $O/ablate.err && echo ABLATE_OK
