#!/bin/bash
# Rehearsal of the multi-rank bench on a one-GPU box: two ranks sharing the card, the all-gather
# over gloo (bench.py --share-gpus --gather gloo); the driver's own N > 1 runs use RCCL over xGMI.
set -u
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
S=scripts/gpu_step.sh
R="python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1"
$S reh_c2 400 $R --master-port 29531 bench.py --gpus 2 --steps 3 --warmup 1 --share-gpus \
  --gather gloo --no-cpu-baseline || exit $?
$S reh_c5 300 $R --master-port 29532 bench.py --gpus 2 --workload c5 --steps 500 --warmup 50 \
  --share-gpus --gather gloo --no-cpu-baseline || exit $?
$S reh_c5fit 300 $R --master-port 29533 bench.py --gpus 2 --workload c5fit --steps 5 --warmup 1 \
  --share-gpus --gather gloo --no-cpu-baseline || exit $?
echo done
