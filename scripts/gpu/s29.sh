#!/bin/bash
# chunk-major stage order in conv_glds2: numerics, per-layer, step bench, L2 counters
cd "$GRAFT_REPO_ROOT" || exit 2
S=scripts/gpu/run_step.sh
$S conv_tests 600 python -u -m pytest tests/test_gpu_conv.py -x -q --timeout 300 --timeout-method thread || exit $?
$S convs 300 python scripts/bench_convs.py --no-ref || exit $?
$S bench_g1 600 python bench.py --steps 20 --warmup 5 || exit $?
export TMPDIR=/tmp
$S pmc_l2 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum GRBM_GUI_ACTIVE --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/pmc29" -o run -- python3 "$GRAFT_REPO_ROOT/scripts/bench_convs.py" --no-ref --layers F4,F9,B2 || exit $?
echo done
