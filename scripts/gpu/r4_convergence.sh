#!/bin/bash
# r4_convergence.sh: training-curve parity of the round-4 default native step (bf16 and fp16) against stock fp32
# PyTorch from one init, 384x512, 400 steps, with declared tolerances -> gpurun_out/convergence_384x512.jsonl
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
S=scripts/gpu/run_step.sh
$S conv 900 python scripts/convergence.py --epochs 50 --train 64 --test 16 --batch 8 --height 384 --width 512 --lr 1e-7 --out gpurun_out/convergence_384x512.jsonl || exit $?
echo done
