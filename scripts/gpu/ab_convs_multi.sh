#!/bin/bash
# Per-layer conv timings of several environment arms, interleaved: ab_convs_multi.sh LAYERS PASSES ROUNDS "ENV1" "ENV2" ...
# -> gpurun_out/arm<i>_<round>.log (read with scripts/dev/arms_report.py)
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
S=scripts/gpu/run_step.sh
L=$1; P=$2; R=$3; shift 3
for r in $(seq $R); do
  i=0
  for arm in "$@"; do
    env $arm $S arm${i}_$r 300 python scripts/bench_convs.py --no-ref --layers "$L" --passes "$P" || exit $?
    i=$((i + 1))
  done
done
echo done
