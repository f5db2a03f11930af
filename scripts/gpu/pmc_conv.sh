#!/bin/bash
# pmc_conv.sh NAME LAYERS [PASSES]: PMC counter passes (each in its own run, no tracing domains) over
# scripts/bench_convs.py for the given layers -> gpurun_out/NAME_{util,wait,inst,l2}/
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
name=$1; L=$2; P=${3:-fwd,dgrad,wgrad}
S=scripts/gpu/run_step.sh
B="python3 $GRAFT_REPO_ROOT/scripts/bench_convs.py --no-ref --layers $L --passes $P --iters 5"
run() {  # run TAG counters...
  tag=$1; shift
  $S ${name}_$tag 120 timeout -s KILL 110 rocprofv3 --pmc "$@" --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/${name}_$tag" -o run -- $B || exit $?
}
run util MfmaUtil LdsBankConflict
run wait SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES
run inst SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_VMEM
run l2 TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE
echo done
