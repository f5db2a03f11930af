#!/bin/bash
# r4_pmc_step.sh: PMC counter passes (each its own run, no tracing domains) over the default training step
# (bench.py, 2 warm-up + 3 steps; counter collection serialises the kernels) -> gpurun_out/pmcstep_{util,wait,inst}/
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
S=scripts/gpu/run_step.sh
B="python3 $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 2 --comm-steps 0"
run() {  # run TAG counters...
  tag=$1; shift
  $S pmcstep_$tag 150 timeout -s KILL 140 rocprofv3 --pmc "$@" --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/pmcstep_$tag" -o run -- $B || exit $?
}
run util MfmaUtil LdsBankConflict
run wait SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES
run inst SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_VMEM
echo done
