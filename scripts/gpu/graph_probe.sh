#!/bin/bash
# graph_probe.sh: eager vs hipGraph replay in bf16 and fp16 (bench lines), plus a kernel trace of each replay mode.
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
S=scripts/gpu/run_step.sh
$S b_bf16_eager 300 python bench.py --steps 30 --warmup 5 || exit $?
$S b_bf16_graph 300 python bench.py --steps 30 --warmup 5 --graph 1 || exit $?
$S b_fp16_eager 300 python bench.py --steps 30 --warmup 5 --dtype fp16 || exit $?
$S b_fp16_graph 300 python bench.py --steps 30 --warmup 5 --dtype fp16 --graph 1 || exit $?
$S p_graph 600 rocprofv3 --kernel-trace --stats -d gpurun_out/p_graph -o step -- python3 bench.py --steps 3 --warmup 2 --comm-steps 0 --graph 1 || exit $?
$S p_eager 600 rocprofv3 --kernel-trace --stats -d gpurun_out/p_eager -o step -- python3 bench.py --steps 3 --warmup 2 --comm-steps 0 || exit $?
grep -h '"metric"' gpurun_out/b_*.log > gpurun_out/graph_probe.jsonl
echo done
