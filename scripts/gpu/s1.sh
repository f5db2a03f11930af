#!/bin/bash
# GPU session 1: toolchain/runtime probe, conv kernel numerics, stock-stack baseline + profile.
cd "$GRAFT_REPO_ROOT" || exit 2
S=scripts/gpu/run_step.sh
$S probe 300 python -c "import torch, can_distributed_pytorch_amd.ops._ext as e; m=e.require(); print('arch', m.arch(), torch.cuda.get_device_name())" || exit $?
$S pytest_gpu 600 python -m pytest tests -m gpu -x -q || exit $?
$S bench_torch_fp32 600 python bench.py --impl torch --dtype fp32 --steps 10 --warmup 3 || exit $?
$S bench_torch_bf16 600 python bench.py --impl torch --dtype bf16 --steps 10 --warmup 3 || exit $?
export TMPDIR=/tmp
$S prof_torch_bf16 600 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof_torch_bf16" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --impl torch --dtype bf16 --steps 3 --warmup 2 || exit $?
echo done
