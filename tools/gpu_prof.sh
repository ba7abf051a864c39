#!/bin/bash
# rocprofv3 kernel-trace stats of one bench config: tools/gpu_prof.sh TAG CONFIG [extra bench args]
set -o pipefail
TAG=${1:-prof}; C=${2:-4}; shift 2
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_c$C -o run -- python bench.py --config $C --steps 5 --warmup 1 --no-cpu-baseline "$@" > $O/bench_c$C.json 2> $O/prof_c$C.err || { tail -20 $O/prof_c$C.err; exit 1; }
f=$(find $O/trace_c$C -name '*kernel_stats.csv' | head -1)
python - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: -float(r['TotalDurationNs']))
for r in rows[:14]:
    n = r['Name']
    n = n[:90]
    print('%8.3f ms avg %8.3f x%4s  %s' % (float(r['TotalDurationNs'])/1e6, float(r['AverageNs'])/1e6, r['Calls'], n))
PY
