#!/bin/bash
# prof_step.sh NAME [bench args...]: kernel-trace profile of a short bench run -> gpurun_out/NAME/
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
name=$1; shift
scripts/gpu/run_step.sh "$name" 600 rocprofv3 --kernel-trace --stats -d "gpurun_out/$name" -o step -- python3 bench.py --steps 3 --warmup 2 --comm-steps 0 "$@"
