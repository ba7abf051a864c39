#!/bin/bash
# LDS bank-conflict counters of the face scan, one --pmc pass
# per workload (SQ counters only, no tracing domain beside --pmc):
#   tools/gpu_sq.sh TAG ["2048:16 512:10"]
set -o pipefail
TAG=${1:-sq}; WL=${2:-"2048:16 512:10"}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$TAG
mkdir -p $O
for w in $WL; do
  S=${w%%:*}; C=${w##*:}
  CTG_PROF_SIZE=$S CTG_PROF_CELL=$C CTG_PROF_ITERS=2 timeout -s KILL 240 rocprofv3 \
      --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_WAVES SQ_BUSY_CYCLES \
      --output-format csv -d $O/sq_$S -o run -- python tools/prof_scan.py boundary > $O/sq_$S.log 2>&1 || { echo "SQ $S FAILED"; tail -5 $O/sq_$S.log; exit 1; }
  python - "$O/sq_$S" <<'PY'
import csv, glob, sys
acc = {}
for f in glob.glob(sys.argv[1] + '/**/*counter_collection.csv', recursive=True):
    for r in csv.DictReader(open(f)):
        if 'k_face_scan' not in r['Kernel_Name']:
            continue
        acc.setdefault(r['Counter_Name'], []).append(float(r['Counter_Value']))
m = {k: max(v) for k, v in acc.items()}   # the launched tile width (the other exits at once)
c, a = m.get('SQ_LDS_BANK_CONFLICT', 0), m.get('SQ_LDS_IDX_ACTIVE', 0)
print('SQ', sys.argv[1], {k: '%.4g' % v for k, v in sorted(m.items())}, 'conflict/active = %.3f' % (c / a if a else -1))
PY
done
