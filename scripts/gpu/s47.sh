#!/bin/bash
# current step profile (kernel trace + stats) for the re-entry baseline
cd "$GRAFT_REPO_ROOT" || exit 2
S=scripts/gpu/run_step.sh
export TMPDIR=/tmp
$S prof_native 600 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof47" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --graph 0 --steps 3 --warmup 2 || exit $?
echo done
