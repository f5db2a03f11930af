#!/bin/bash
# r4_confirm.sh: every GPU test with the current defaults (stop on failure), then the step with the defaults vs the
# previous tap settings (interleaved), the bench lines (hipGraph with the one-queue setting, fp16, 1080x1920) and a
# kernel trace of the default step.
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
S=scripts/gpu/run_step.sh
$S tests 1100 python -u -m pytest tests -m gpu -x -q -rf --timeout 240 --timeout-method thread -p no:cacheprovider || exit $?
grep -q "failed\|error" gpurun_out/tests.log && { echo "tests failed: stop"; exit 1; }
for r in 1 2 3; do
  $S step_def_$r 300 python bench.py --steps 30 --warmup 5 || exit $?
  CANNET_DISPATCH=wgrad_tap_adb=0 $S step_noadb_$r 300 python bench.py --steps 30 --warmup 5 || exit $?
  CANNET_DISPATCH=wgrad_tap=2,wgrad_tap_adb=0 $S step_tap2_$r 300 python bench.py --steps 30 --warmup 5 || exit $?
  # (profiles/r4/ab_confirm.txt also has wgrad_tap_ks=1 / bwd_priority=1 arms, run at commit 7a9a511; both removed)
  CANNET_DISPATCH=rring128=2 $S step_r128_$r 300 python bench.py --steps 30 --warmup 5 || exit $?
done
$S b_default 300 python bench.py || exit $?
$S b_graph 300 python bench.py --steps 30 --warmup 5 --graph 1 || exit $?
$S b_fp16 300 python bench.py --steps 30 --warmup 5 --dtype fp16 || exit $?
$S b_fp16_graph 300 python bench.py --steps 30 --warmup 5 --graph 1 --dtype fp16 || exit $?
$S b_1080_b8 300 python bench.py --steps 20 --warmup 3 --batch 8 --height 1080 --width 1920 || exit $?
$S b_b32 300 python bench.py --steps 10 --warmup 3 --batch 32 || exit $?
grep -h '"metric"' gpurun_out/b_*.log > gpurun_out/bench_confirm.jsonl
$S p_eager 600 rocprofv3 --kernel-trace --stats -d gpurun_out/p_eager -o step -- python3 bench.py --steps 3 --warmup 2 --comm-steps 0 || exit $?
DEBUG_HIP_FORCE_GRAPH_QUEUES=1 $S p_graph 600 rocprofv3 --kernel-trace --stats -d gpurun_out/p_graph -o step -- python3 bench.py --steps 3 --warmup 2 --comm-steps 0 --graph 1 || exit $?
echo done
