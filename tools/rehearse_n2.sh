#!/bin/bash
# bench.py's N>1 path on the one-GPU box: 2 ranks on cuda:0, gloo exchange.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-n2}
mkdir -p $O
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 \
    bench.py --gpus 2 --steps 5 --warmup 2 --backend gloo --device 0 ${2:-} > $O/bench_n2.json 2> $O/bench_n2.err && echo N2_OK && cat $O/bench_n2.json
