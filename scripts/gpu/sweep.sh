#!/bin/bash
# Config #4/#5 evidence: per-GPU batch sweep at 768x1024, 1080x1920 at batch 8, fp16, hipGraph step,
# and a kernel trace of the graph replay (does the captured step overlap the weight-gradient stream?).
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
S=scripts/gpu/run_step.sh
for b in 8 16 32; do
  $S sweep_b$b 600 python bench.py --batch $b --steps 10 --warmup 3 || exit $?
done
$S sweep_1080 600 python bench.py --batch 8 --height 1080 --width 1920 --steps 10 --warmup 3 || exit $?
$S sweep_fp16 600 python bench.py --dtype fp16 --steps 20 --warmup 5 || exit $?
$S sweep_graph 600 python bench.py --graph 1 --steps 20 --warmup 5 || exit $?
$S sweep_eager 600 python bench.py --graph 0 --steps 20 --warmup 5 || exit $?
scripts/gpu/prof_step.sh prof_graph --graph 1 || exit $?
echo done
