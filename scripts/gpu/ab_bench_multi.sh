#!/bin/bash
# Step bench of several environment arms, interleaved: ab_bench_multi.sh ROUNDS "ENV1" "ENV2" ...
# -> gpurun_out/barm<i>_<round>.log (read with scripts/dev/arms_report.py --bench)
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
S=scripts/gpu/run_step.sh
R=$1; shift
for r in $(seq $R); do
  i=0
  for arm in "$@"; do
    env $arm $S barm${i}_$r 300 python bench.py --steps 30 --warmup 5 || exit $?
    i=$((i + 1))
  done
done
echo done
