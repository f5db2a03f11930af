#!/bin/bash
# ragged_train.sh: the reference's own workload (train.py, batch 1 per GPU, variable-size JPEGs, reference
# train.py:177 / model/CrowdDataset.py:53-62) on locally written ShanghaiTech-layout sets, against the fixed
# 768x1024 set, plus batch 8 of one ragged size and the 1080x1920 bench line.  JSONL -> gpurun_out/ragged/.
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
S=scripts/gpu/run_step.sh
mkdir -p gpurun_out/ragged
timeout 600 python scripts/make_jpeg_set.py --root /tmp/sha_mixed --train 160 --test 16 --mixed --workers 12 > gpurun_out/ragged/mk1.log 2>&1 || exit $?
timeout 600 python scripts/make_jpeg_set.py --root /tmp/sha_768 --train 160 --test 16 --height 768 --width 1024 --workers 12 > gpurun_out/ragged/mk2.log 2>&1 || exit $?
timeout 600 python scripts/make_jpeg_set.py --root /tmp/sha_680 --train 160 --test 16 --height 680 --width 1016 --workers 12 > gpurun_out/ragged/mk3.log 2>&1 || exit $?
T="python train.py --epochs 3 --eval-every 100 --show False --wandb False --num-workers 12 --seed 0"
$S t_mixed_b1 600 $T --data_root /tmp/sha_mixed --batch-size 1 --checkpoint-dir /tmp/ck1 --log-jsonl gpurun_out/ragged/train_mixed_b1.jsonl || exit $?
$S t_768_b1 600 $T --data_root /tmp/sha_768 --batch-size 1 --checkpoint-dir /tmp/ck2 --log-jsonl gpurun_out/ragged/train_768x1024_b1.jsonl || exit $?
$S t_680_b8 600 $T --data_root /tmp/sha_680 --batch-size 8 --checkpoint-dir /tmp/ck3 --log-jsonl gpurun_out/ragged/train_680x1016_b8.jsonl || exit $?
$S t_768_b8 600 $T --data_root /tmp/sha_768 --batch-size 8 --checkpoint-dir /tmp/ck4 --log-jsonl gpurun_out/ragged/train_768x1024_b8.jsonl || exit $?
$S b_1080 400 python bench.py --steps 20 --warmup 3 --height 1080 --width 1920 || exit $?
$S b_680 400 python bench.py --steps 20 --warmup 3 --height 680 --width 1016 || exit $?
grep -h '"metric"' gpurun_out/b_1080.log gpurun_out/b_680.log > gpurun_out/ragged/bench_ragged.jsonl
echo done
