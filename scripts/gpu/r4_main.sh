#!/bin/bash
# r4_main.sh: row-ring / pool conv tests first (stop on ANY failure: a wrong row-ring DMA address faults the GPU),
# then every GPU test, then the bench lines of r4_tests_big.sh.
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
S=scripts/gpu/run_step.sh
K="test_conv_pool_fwd_fused or test_row_ring_conv_bitwise or test_conv_fwd or test_image_chunked_launches"
$S rr_tests 400 python -u -m pytest tests/test_gpu_conv.py -x -q -rf --timeout 120 --timeout-method thread -p no:cacheprovider -k "$K" || exit $?
grep -q " passed" gpurun_out/rr_tests.log && ! grep -q "failed\|error" gpurun_out/rr_tests.log || { echo "rr_tests failed: stop"; exit 1; }
$S tests 1100 python -u -m pytest tests -m gpu -x -q -rf --timeout 240 --timeout-method thread -p no:cacheprovider || exit $?
grep -q "failed\|error" gpurun_out/tests.log && { echo "tests failed: stop"; exit 1; }
$S b_default 300 python bench.py --steps 30 --warmup 5 || exit $?
$S b_b64 400 python bench.py --steps 6 --warmup 2 --batch 64 || exit $?
$S b_1080_b24 400 python bench.py --steps 6 --warmup 2 --batch 24 --height 1080 --width 1920 || exit $?
$S b_1080_b8 300 python bench.py --steps 20 --warmup 3 --batch 8 --height 1080 --width 1920 || exit $?
$S b_graph 300 python bench.py --steps 30 --warmup 5 --graph 1 || exit $?
$S b_fp16_graph 300 python bench.py --steps 30 --warmup 5 --graph 1 --dtype fp16 || exit $?
grep -h '"metric"' gpurun_out/b_*.log > gpurun_out/bench_main.jsonl
echo done
