set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r1
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/r1/pytest_gpu.log 2>&1 && echo PYTEST_OK &&
timeout -k 10 200 python bench.py --steps 10 --warmup 3 > gpurun_out/r1/bench.json 2> gpurun_out/r1/bench.err && cat gpurun_out/r1/bench.json &&
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r1/prof -o run -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r1/bench_prof.json 2> gpurun_out/r1/prof.err && echo PROF_OK
