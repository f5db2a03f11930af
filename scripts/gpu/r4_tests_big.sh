#!/bin/bash
# r4_tests_big.sh: every GPU test, then the config-#4 HBM-sizing bench lines (batch 64 at 768x1024, batch 24 at
# 1080x1920: beyond the old 32-bit per-launch limit, so the image-chunked launches run), per-layer conv timings,
# hipGraph replay under the HIP runtime's graph-queue knobs, and kernel traces of the eager and replayed step.
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
S=scripts/gpu/run_step.sh
$S tests 1100 python -u -m pytest tests -m gpu -x -q -rf --timeout 240 --timeout-method thread -p no:cacheprovider || exit $?
$S b_default 300 python bench.py --steps 30 --warmup 5 || exit $?
$S b_b64 400 python bench.py --steps 6 --warmup 2 --batch 64 || exit $?
$S b_1080_b24 400 python bench.py --steps 6 --warmup 2 --batch 24 --height 1080 --width 1920 || exit $?
$S b_graph 300 python bench.py --steps 30 --warmup 5 --graph 1 || exit $?
DEBUG_HIP_FORCE_GRAPH_QUEUES=4 $S b_graph_q4 300 python bench.py --steps 30 --warmup 5 --graph 1 || exit $?
DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 $S b_graph_nopc 300 python bench.py --steps 30 --warmup 5 --graph 1 || exit $?
grep -h '"metric"' gpurun_out/b_*.log > gpurun_out/bench_big.jsonl
$S convs 600 python scripts/bench_convs.py --no-ref --iters 20 || exit $?
$S p_eager 600 rocprofv3 --kernel-trace --stats -d gpurun_out/p_eager -o step -- python3 bench.py --steps 3 --warmup 2 --comm-steps 0 || exit $?
$S p_graph 600 rocprofv3 --kernel-trace --stats -d gpurun_out/p_graph -o step -- python3 bench.py --steps 3 --warmup 2 --comm-steps 0 --graph 1 || exit $?
echo done
