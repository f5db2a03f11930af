#!/bin/bash
# Full GPU checkpoint: every GPU test, smoke(), bench lines (eager x2, hipGraph, fp16), one kernel-trace profile.
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
S=scripts/gpu/run_step.sh
$S tests 1100 python -u -m pytest tests -m gpu -x -q -rf --timeout 240 --timeout-method thread || exit $?
$S smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit $?
$S bench_e1 300 python bench.py --steps 30 --warmup 5 || exit $?
$S bench_graph 300 python bench.py --steps 30 --warmup 5 --graph 1 || exit $?
$S bench_fp16 300 python bench.py --steps 30 --warmup 5 --dtype fp16 || exit $?
$S bench_e2 300 python bench.py --steps 30 --warmup 5 || exit $?
$S prof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_full -o step -- python3 bench.py --steps 3 --warmup 2 --comm-steps 0 || exit $?
echo done
