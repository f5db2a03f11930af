#!/bin/bash
# batched-pack check + PMC counter passes on the v2 kernels (counters in their own runs, no tracing domains)
cd "$GRAFT_REPO_ROOT" || exit 2
S=scripts/gpu/run_step.sh
$S exec_tests 900 python -m pytest tests/test_gpu_executor.py -q -rf || exit $?
export TMPDIR=/tmp
$S pmc_util 600 rocprofv3 --pmc MfmaUtil LdsBankConflict --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/pmc24a" -o run -- python3 "$GRAFT_REPO_ROOT/scripts/bench_convs.py" --no-ref --layers F2,F4,F9,B2 || exit $?
$S pmc_wait 600 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/pmc24b" -o run -- python3 "$GRAFT_REPO_ROOT/scripts/bench_convs.py" --no-ref --layers F2,F9,B2 || exit $?
$S pmc_lds 600 rocprofv3 --pmc SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_MFMA --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/pmc24c" -o run -- python3 "$GRAFT_REPO_ROOT/scripts/bench_convs.py" --no-ref --layers F2,F9,B2 || exit $?
echo done
