#!/bin/bash
# A/B of an environment switch on the step bench: ab_env.sh "VAR=value [VAR2=value]" [rounds]
# interleaved rounds on one box (a single pair is within DVFS/thermal noise); read with scripts/dev/ab_report.py.
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
S=scripts/gpu/run_step.sh
R=${2:-3}
for r in $(seq $R); do
  $S ab_bench_old_$r 300 python bench.py --steps 30 --warmup 5 || exit $?
  env $1 $S ab_bench_new_$r 300 python bench.py --steps 30 --warmup 5 || exit $?
done
echo done
