#!/bin/bash
# hipGraph with two streams: do the side-stream weight gradients run concurrently inside a graph?
cd "$GRAFT_REPO_ROOT" || exit 2
S=scripts/gpu/run_step.sh
$S eager_side 600 python bench.py --steps 30 --warmup 5 --graph 0 || exit $?
$S graph_side 600 python bench.py --steps 30 --warmup 5 --graph 1 || exit $?
DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 $S graph_nopkt 600 python bench.py --steps 30 --warmup 5 --graph 1 || exit $?
DEBUG_HIP_FORCE_GRAPH_QUEUES=4 $S graph_q4 600 python bench.py --steps 30 --warmup 5 --graph 1 || exit $?
$S eager_side2 600 python bench.py --steps 30 --warmup 5 --graph 0 || exit $?
export TMPDIR=/tmp
$S prof_side 600 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof39" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --graph 0 --steps 3 --warmup 2 || exit $?
echo done
