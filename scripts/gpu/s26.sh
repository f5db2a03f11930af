#!/bin/bash
# re-entry check: full GPU tier, step bench, per-layer convs
cd "$GRAFT_REPO_ROOT" || exit 2
S=scripts/gpu/run_step.sh
$S gpu_tests 900 python -u -m pytest tests -m gpu -x -q -rf --timeout 300 --timeout-method thread || exit $?
$S bench_g1 600 python bench.py --steps 20 --warmup 5 || exit $?
$S convs 300 python scripts/bench_convs.py --no-ref || exit $?
echo done
