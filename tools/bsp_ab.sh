set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/bsp1; mkdir -p $O
CTG_BUCKET_SORT_PAIRS=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_blocks.py tests/test_gpu_fullsize.py -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -1 $O/pytest.log; grep FAILED $O/pytest.log | head -5; [ $rc -eq 0 ] || exit 1
timeout -k 10 600 python tools/ab_variants.py b1024c5,nn1024,b2048 base base@CTG_BUCKET_SORT_PAIRS=1 > $O/ab.jsonl 2> $O/ab.err || { tail -5 $O/ab.err; exit 1; }
cat $O/ab.jsonl
