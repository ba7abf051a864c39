cd "$GRAFT_REPO_ROOT" || exit 1
bash tools/gpu_tests.sh r3codec && \
CTG_BLOCK_BATCH_BYTES=536870912 timeout -k 10 300 python bench.py --config 0 --steps 3 --warmup 1 > gpurun_out/r3codec/bench_c0_512m.json 2> gpurun_out/r3codec/bench_c0_512m.err && \
CTG_BLOCK_BATCH_BYTES=134217728 timeout -k 10 300 python bench.py --config 0 --steps 3 --warmup 1 > gpurun_out/r3codec/bench_c0_128m.json 2> gpurun_out/r3codec/bench_c0_128m.err
