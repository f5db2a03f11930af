#!/bin/bash
# r4_serial.sh: weight gradients on the side stream (default) vs in order on the compute stream (wgrad_stream=0)
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
S=scripts/gpu/run_step.sh
for r in 1 2 3; do
  $S step_base_$r 300 python bench.py --steps 30 --warmup 5 || exit $?
  CANNET_DISPATCH=wgrad_stream=0 $S step_serial_$r 300 python bench.py --steps 30 --warmup 5 || exit $?
done
echo done
