#!/bin/bash
# Round-4 multi-GPU step costs on the one-GPU box: the default bench line
# (configs[2]), the RCCL world-1 distributed path (configs[1], [2]) and the
# N=2 rehearsal (both ranks on cuda:0, gloo wire) of configs[1] and [2];
# then the drop-in job-process exit probe (tools/exit_cost.py).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r4d}
mkdir -p $O
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
cat $O/bench.json
for c in 1 2; do
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
    --master-port 2954$c bench.py --config $c --gpus 1 --dist-path --steps 20 --warmup 3 --no-cpu-baseline \
    > $O/bench_dist1_c$c.json 2> $O/bench_dist1_c$c.err || { tail -5 $O/bench_dist1_c$c.err; exit 1; }
  cat $O/bench_dist1_c$c.json
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 2955$c bench.py --config $c --gpus 2 --steps 10 --warmup 2 --backend gloo --device 0 \
    --no-cpu-baseline > $O/bench_n2_c$c.json 2> $O/bench_n2_c$c.err || { tail -5 $O/bench_n2_c$c.err; exit 1; }
  cat $O/bench_n2_c$c.json
done
timeout -k 10 400 python tools/exit_cost.py > $O/exit_cost.jsonl 2> $O/exit_cost.err || { tail -5 $O/exit_cost.err; exit 1; }
cat $O/exit_cost.jsonl
echo R4_DIST_DONE
