#!/bin/bash
# Per-phase wall time of the world-1 RCCL distributed step (CTG_DIST_DEBUG=1:
# a device sync after each phase) at configs[1].
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r4dp}
mkdir -p $O
unset CTG_LIB
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
  --master-port 29561 bench.py --config 1 --gpus 1 --dist-path --steps 20 --warmup 3 --no-cpu-baseline \
  > $O/dist1_plain.json 2> $O/dist1_plain.err || { tail -5 $O/dist1_plain.err; exit 1; }
cat $O/dist1_plain.json
CTG_DIST_DEBUG=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
  --master-addr 127.0.0.1 --master-port 29562 bench.py --config 1 --gpus 1 --dist-path --steps 20 --warmup 3 \
  --no-cpu-baseline > $O/dist1_debug.json 2> $O/dist1_debug.err || { tail -5 $O/dist1_debug.err; exit 1; }
python tools/dist_phases.py $O/dist1_debug.err
echo R4_DISTPH_DONE
