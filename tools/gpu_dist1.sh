#!/bin/bash
# World-1 RCCL step (bench.py --dist-path) beside the local call, per config:
#   tools/gpu_dist1.sh TAG "configs"   (+ one --write-output run of the first config)
set -o pipefail
TAG=${1:-dist1}; CFGS=${2:-"1 2"}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$TAG
mkdir -p $O
port=29533
for c in $CFGS; do
  timeout -k 10 300 python bench.py --config $c --steps 20 --warmup 3 --no-cpu-baseline > $O/local_c$c.json 2> $O/local_c$c.err || { echo "LOCAL $c FAILED"; tail -5 $O/local_c$c.err; exit 1; }
  port=$((port+1))
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port $port \
      bench.py --gpus 1 --dist-path --config $c --steps 20 --warmup 3 --no-cpu-baseline > $O/dist1_c$c.json 2> $O/dist1_c$c.err || { echo "DIST1 $c FAILED"; tail -5 $O/dist1_c$c.err; exit 1; }
  python - $O $c <<'PY'
import json, sys
o, c = sys.argv[1], sys.argv[2]
ld = lambda f: json.loads([l for l in open(f) if l.startswith('{')][-1])
a, b = ld('%s/local_c%s.json' % (o, c)), ld('%s/dist1_c%s.json' % (o, c))
print('C%s local %.4f ms  world-1 %.4f ms  ratio %.3f' % (c, a['ms_per_step'], b['ms_per_step'], b['ms_per_step'] / a['ms_per_step']))
PY
done
c=${CFGS%% *}
port=$((port+1))
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port $port \
    bench.py --gpus 1 --dist-path --config $c --steps 5 --warmup 1 --no-cpu-baseline --write-output /tmp/ctg_out_$TAG > $O/dist1_out_c$c.json 2> $O/dist1_out_c$c.err || { echo "OUTPUT FAILED"; tail -5 $O/dist1_out_c$c.err; exit 1; }
python -c "import json; d=json.loads([l for l in open('$O/dist1_out_c$c.json') if l.startswith('{')][-1]); print('OUTPUT', d.get('output'))"
rm -rf /tmp/ctg_out_$TAG
