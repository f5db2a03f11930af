#!/bin/bash
# pmc_ab.sh NAME "VAR=value" LAYERS PASSES: two PMC counter passes over scripts/bench_convs.py, each run once with the
# switch off and once on (each its own rocprofv3 run, no tracing domains) -> gpurun_out/NAME_{off,on}_{a,b}/
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
name=$1; SW=$2; L=$3; P=$4
S=scripts/gpu/run_step.sh
B="python3 $GRAFT_REPO_ROOT/scripts/bench_convs.py --no-ref --layers $L --passes $P --iters 5"
run() {  # run TAG counters...
  tag=$1; shift
  $S ${name}_off_$tag 120 timeout -s KILL 110 rocprofv3 --pmc "$@" --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/${name}_off_$tag" -o run -- $B || exit $?
  env $SW $S ${name}_on_$tag 120 timeout -s KILL 110 rocprofv3 --pmc "$@" --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/${name}_on_$tag" -o run -- $B || exit $?
}
run a SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_MFMA SQ_INSTS_VMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES
run b SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU GRBM_GUI_ACTIVE
echo done
