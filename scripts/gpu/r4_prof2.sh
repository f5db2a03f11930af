#!/bin/bash
# r4_prof2.sh: kernel traces of the isolated weight-gradient layers (bench_convs --passes wgrad: tap kernels and
# their slab reductions one at a time) and of the training step at the current defaults.
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
S=scripts/gpu/run_step.sh
$S prof_wgrad 300 rocprofv3 --kernel-trace -d gpurun_out/prof_wgrad -o wg -- python3 scripts/bench_convs.py --no-ref --passes wgrad --iters 3 || exit $?
$S prof_step 300 rocprofv3 --kernel-trace -d gpurun_out/prof_step -o step -- python3 bench.py --steps 3 --warmup 2 || exit $?
echo done
