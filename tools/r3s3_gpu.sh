#!/bin/bash
# Session-3 GPU step: full GPU suite (RCCL world-1 exchange, sorted_runs parity),
# the N=1 distributed-path line over RCCL, A/B of sorted_runs vs rocPRIM RLE.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-s3b}
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
tail -1 $O/pytest_gpu.log; grep FAILED $O/pytest_gpu.log | head -5; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
  --master-port 29533 bench.py --gpus 1 --dist-path --steps 20 --warmup 3 > $O/bench_dist1.json 2> $O/bench_dist1.err || { tail -5 $O/bench_dist1.err; exit 1; }
cat $O/bench_dist1.json
timeout -k 10 600 python tools/ab_variants.py b1024c5,b512 base base@CTG_SORTED_RUNS=1 > $O/ab.jsonl 2> $O/ab.err || { tail -5 $O/ab.err; exit 1; }
cat $O/ab.jsonl
