#!/bin/bash
# r4_convergence2.sh: the convergence protocol of r4_convergence.sh for two more seeds (initialisation and batch order),
# with stock PyTorch bf16 autocast as the 16-bit yardstick -> gpurun_out/convergence_384x512_s{1,2}.jsonl
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
S=scripts/gpu/run_step.sh
for sd in 1 2; do
  $S conv_s$sd 900 python scripts/convergence.py --epochs 50 --train 64 --test 16 --batch 8 --height 384 --width 512 --lr 1e-7 --seed $sd --out gpurun_out/convergence_384x512_s$sd.jsonl || exit $?
done
echo done
