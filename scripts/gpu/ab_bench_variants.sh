#!/bin/bash
# Step bench of several (tree, environment) arms, interleaved on one box:
#   ab_bench_variants.sh ROUNDS "DIR|ENV" ...   -> gpurun_out/barm<i>_<round>.log (scripts/dev/arms_report.py)
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
S=scripts/gpu/run_step.sh
R=$1; shift
for r in $(seq $R); do
  i=0
  for arm in "$@"; do
    d=${arm%%|*}; e=${arm#*|}
    env $e $S barm${i}_$r 300 python $d/bench.py --steps 30 --warmup 5 || exit $?
    i=$((i + 1))
  done
done
echo done
