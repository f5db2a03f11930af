#!/bin/bash
# r4_final.sh: round-end confirmation on the final tree: every GPU test (stop on failure), the default step three
# times, the bench lines (hipGraph one-queue, fp16, fp16 + graph, 1080x1920 batch 8, batch 32) and a kernel trace of
# the default step.
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
S=scripts/gpu/run_step.sh
$S tests 1100 python -u -m pytest tests -m gpu -x -q -rf --timeout 240 --timeout-method thread -p no:cacheprovider || exit $?
grep -q "failed\|error" gpurun_out/tests.log && { echo "tests failed: stop"; exit 1; }
for r in 1 2 3; do
  $S b_default_$r 300 python bench.py --steps 30 --warmup 5 || exit $?
done
$S b_graph 300 python bench.py --steps 30 --warmup 5 --graph 1 || exit $?
$S b_fp16 300 python bench.py --steps 30 --warmup 5 --dtype fp16 || exit $?
$S b_fp16_graph 300 python bench.py --steps 30 --warmup 5 --graph 1 --dtype fp16 || exit $?
$S b_1080_b8 300 python bench.py --steps 20 --warmup 3 --batch 8 --height 1080 --width 1920 || exit $?
$S b_b32 300 python bench.py --steps 10 --warmup 3 --batch 32 || exit $?
grep -h '"metric"' gpurun_out/b_*.log > gpurun_out/bench_final.jsonl
$S p_eager 600 rocprofv3 --kernel-trace -d gpurun_out/p_eager -o step -- python3 bench.py --steps 3 --warmup 2 --comm-steps 0 || exit $?
echo done
