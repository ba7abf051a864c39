#!/bin/bash
# Round-4 GPU step: the GPU suite (incl. the 2048^3 tests against the torch
# enumeration), smoke(), the default bench line (configs[2]) with its CPU
# baseline, the world-1 RCCL distributed path of configs[1] and [2] under
# rocprofv3 --kernel-trace --stats (where the multi-GPU step's fixed cost goes).
# usage: tools/r4_gpu.sh <tag> [skip-tests]
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r4a}
mkdir -p $O
if [ "$2" != skip-tests ]; then
  timeout -k 10 700 python -u -m pytest tests -m gpu -v --timeout 600 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
  tail -1 $O/pytest_gpu.log; grep FAILED $O/pytest_gpu.log | head -5; [ $rc -eq 0 ] || exit 1
  timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 1; }
  cat $O/smoke.log
fi
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
cat $O/bench.json
for c in 1 2; do
  # one rank without a launcher (rocprofv3 must sit directly in front of the program):
  # the env:// rendezvous variables torch.distributed.run would set
  MASTER_ADDR=127.0.0.1 MASTER_PORT=2953$c RANK=0 LOCAL_RANK=0 WORLD_SIZE=1 \
    timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_dist_c$c -o run -- \
    python bench.py --config $c --gpus 1 --dist-path --steps 10 --warmup 2 --no-cpu-baseline \
    > $O/bench_dist_c$c.json 2> $O/bench_dist_c$c.err || { tail -5 $O/bench_dist_c$c.err; exit 1; }
  cat $O/bench_dist_c$c.json
done
echo R4_GPU_DONE
