#!/bin/bash
# Real-format input pipeline at speed + training-curve parity:
#  1) a local 768x1024 JPEG set (ShanghaiTech layout), 2) train.py on it (decode in workers, packed H2D,
#  one preprocessing launch per batch), JSONL log, 3) native bf16 vs torch fp32 curves (scripts/convergence.py)
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
S=scripts/gpu/run_step.sh
$S synth_test 300 python -u -m pytest tests/test_gpu_components.py -k "synthetic or packed" -x -q --timeout 120 || exit $?
$S make_set 600 python -u scripts/make_jpeg_set.py --root /tmp/sha_synth --train 768 --test 32 --workers 16 || exit $?
$S train_jpeg 900 python -u train.py --data_root /tmp/sha_synth --epochs 3 --batch-size 8 --num-workers 16 \
   --show false --wandb false --eval-every 3 --checkpoint-dir /tmp/ckpt --log-jsonl gpurun_out/train_jpeg.jsonl || exit $?

echo done
