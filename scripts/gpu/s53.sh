#!/bin/bash
# full GPU suite + smoke + bench + per-kernel step profile of the committed tree
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
S=scripts/gpu/run_step.sh
$S gpu_tests 900 python -u -m pytest tests -m gpu -x -q -rf --timeout 240 --timeout-method thread || exit $?
$S smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit $?
for r in 1 2; do
  $S bench$r 600 python bench.py --steps 30 --warmup 5 || exit $?
done
$S prof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o step -- python3 bench.py --graph 0 --steps 3 --warmup 2 || exit $?
echo done
