#!/bin/bash
# r4_check.sh: every GPU test, the default 1-GPU bench line, the eager/graph x bf16/fp16 bench lines and a kernel trace
# of the default step.  Results under gpurun_out/.
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
S=scripts/gpu/run_step.sh
$S tests 1100 python -u -m pytest tests -m gpu -x -q -rf --timeout 240 --timeout-method thread -p no:cacheprovider || exit $?
$S b_bf16_eager 300 python bench.py --steps 30 --warmup 5 || exit $?
$S b_bf16_graph 300 python bench.py --steps 30 --warmup 5 --graph 1 || exit $?
$S b_fp16_eager 300 python bench.py --steps 30 --warmup 5 --dtype fp16 || exit $?
$S b_fp16_graph 300 python bench.py --steps 30 --warmup 5 --dtype fp16 --graph 1 || exit $?
grep -h '"metric"' gpurun_out/b_*.log > gpurun_out/bench_modes.jsonl
$S p_eager 600 rocprofv3 --kernel-trace --stats -d gpurun_out/p_eager -o step -- python3 bench.py --steps 3 --warmup 2 --comm-steps 0 || exit $?
$S p_graph 600 rocprofv3 --kernel-trace --stats -d gpurun_out/p_graph -o step -- python3 bench.py --steps 3 --warmup 2 --comm-steps 0 --graph 1 || exit $?
echo done
