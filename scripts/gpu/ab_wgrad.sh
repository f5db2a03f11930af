#!/bin/bash
# A/B: isolated per-layer conv times, old (ab_old/) vs new build, interleaved rounds on one box; then the step
# bench, interleaved rounds too (a single bench pair is within DVFS/thermal noise).
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
S=scripts/gpu/run_step.sh
L=${AB_LAYERS:-F6,F9,B1,B2}
R=${AB_ROUNDS:-2}
for r in $(seq $R); do
  $S ab_old_$r 300 python ab_old/scripts/bench_convs.py --no-ref --layers $L || exit $?
  $S ab_new_$r 300 python scripts/bench_convs.py --no-ref --layers $L || exit $?
done
for r in 1 2 3; do
  $S ab_bench_old_$r 300 python ab_old/bench.py --steps 30 --warmup 5 || exit $?
  $S ab_bench_new_$r 300 python bench.py --steps 30 --warmup 5 || exit $?
done
echo done
