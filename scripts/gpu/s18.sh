#!/bin/bash
# PMC counter passes on representative conv layers (counters in their own runs, no tracing domains)
cd "$GRAFT_REPO_ROOT" || exit 2
S=scripts/gpu/run_step.sh
export TMPDIR=/tmp
$S pmc_mfma 600 rocprofv3 --pmc MfmaUtil LdsBankConflict --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/pmc1" -o run -- python3 "$GRAFT_REPO_ROOT/scripts/bench_convs.py" --no-ref --layers F2,F4,F9,B2 || exit $?
$S pmc_mem 600 rocprofv3 --pmc FETCH_SIZE TCC_HIT_sum TCC_MISS_sum --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/pmc2" -o run -- python3 "$GRAFT_REPO_ROOT/scripts/bench_convs.py" --no-ref --layers F2,F4,F9,B2 || exit $?
$S bench_native 600 python bench.py --steps 20 --warmup 3 || exit $?
$S prof_native 600 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof_native18" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --graph 0 --steps 3 --warmup 2 || exit $?
echo done
