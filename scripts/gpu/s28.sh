#!/bin/bash
# 2-rank DP native-step test + L2 hit-rate counters of the big conv kernels
cd "$GRAFT_REPO_ROOT" || exit 2
S=scripts/gpu/run_step.sh
$S dp_test 300 python -u -m pytest tests/test_gpu_dp.py -x -v --timeout 240 --timeout-method thread || exit $?
export TMPDIR=/tmp
$S pmc_l2 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum GRBM_GUI_ACTIVE --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/pmc28" -o run -- python3 "$GRAFT_REPO_ROOT/scripts/bench_convs.py" --no-ref --layers F2,F4,F9,B2 || exit $?
echo done
