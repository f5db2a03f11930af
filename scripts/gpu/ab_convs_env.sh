#!/bin/bash
# Per-layer conv A/B of an environment switch: ab_convs_env.sh "VAR=value" LAYERS PASSES [rounds]
# interleaved rounds on one box (gpurun_out/ab_old_*.log = switch off, ab_new_*.log = on); read with
# scripts/dev/ab_report.py.
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
S=scripts/gpu/run_step.sh
R=${4:-2}
for r in $(seq $R); do
  $S ab_old_$r 300 python scripts/bench_convs.py --no-ref --layers "$2" --passes "$3" || exit $?
  env $1 $S ab_new_$r 300 python scripts/bench_convs.py --no-ref --layers "$2" --passes "$3" || exit $?
done
echo done
