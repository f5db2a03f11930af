#!/bin/bash
# Per-layer conv timings of several (tree, environment) arms, interleaved on one box:
#   ab_convs_variants.sh LAYERS PASSES ROUNDS "DIR|ENV" ...   (DIR "." = this tree, ab_<name> = a variant build,
#   scripts/gpu/ab_variant_build.sh) -> gpurun_out/arm<i>_<round>.log (scripts/dev/arms_report.py)
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
S=scripts/gpu/run_step.sh
L=$1; P=$2; R=$3; shift 3
for r in $(seq $R); do
  i=0
  for arm in "$@"; do
    d=${arm%%|*}; e=${arm#*|}
    env $e $S arm${i}_$r 300 python $d/scripts/bench_convs.py --no-ref --layers "$L" --passes "$P" || exit $?
    i=$((i + 1))
  done
done
echo done
