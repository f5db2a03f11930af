#!/bin/bash
# A/B of the step bench only: ab_old/ (scripts/gpu/ab_old.sh) vs the working tree, interleaved rounds on one box.
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
S=scripts/gpu/run_step.sh
R=${1:-3}
shift
for r in $(seq $R); do
  $S ab_bench_old_$r 300 python ab_old/bench.py --steps 30 --warmup 5 "$@" || exit $?
  $S ab_bench_new_$r 300 python bench.py --steps 30 --warmup 5 "$@" || exit $?
done
echo done
