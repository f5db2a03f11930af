#!/bin/bash
# r4_full.sh: every GPU test (stop on failure), the bench lines (default, hipGraph bf16 / fp16, 1080x1920 b8), a
# kernel trace of the eager and the graph-replayed step, and PMC passes over the per-layer conv / weight-gradient
# kernels.
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
S=scripts/gpu/run_step.sh
$S tests 1100 python -u -m pytest tests -m gpu -x -q -rf --timeout 240 --timeout-method thread -p no:cacheprovider || exit $?
grep -q "failed\|error" gpurun_out/tests.log && { echo "tests failed: stop"; exit 1; }
$S b_default 300 python bench.py --steps 30 --warmup 5 || exit $?
$S b_default2 300 python bench.py --steps 30 --warmup 5 || exit $?
$S b_graph 300 python bench.py --steps 30 --warmup 5 --graph 1 || exit $?
$S b_fp16 300 python bench.py --steps 30 --warmup 5 --dtype fp16 || exit $?
$S b_fp16_graph 300 python bench.py --steps 30 --warmup 5 --graph 1 --dtype fp16 || exit $?
$S b_1080_b8 300 python bench.py --steps 20 --warmup 3 --batch 8 --height 1080 --width 1920 || exit $?
grep -h '"metric"' gpurun_out/b_*.log > gpurun_out/bench_full.jsonl
$S p_eager 600 rocprofv3 --kernel-trace --stats -d gpurun_out/p_eager -o step -- python3 bench.py --steps 3 --warmup 2 --comm-steps 0 || exit $?
$S p_graph 600 rocprofv3 --kernel-trace --stats -d gpurun_out/p_graph -o step -- python3 bench.py --steps 3 --warmup 2 --comm-steps 0 --graph 1 || exit $?
bash scripts/gpu/pmc_conv.sh pmc F2,F3,F4,F5,F6,F9,B1,B2 || exit $?
echo done
