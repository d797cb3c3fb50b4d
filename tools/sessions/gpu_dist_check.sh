#!/bin/bash
# The multi-GPU launch path on one box: bench.py under torch.distributed.run (one rank, RCCL
# process group, per-rank hipRTC compile before the timed region) for the C5 flocking preset and the
# default C2 line.  The driver's N=2/4/8 runs use this same code path on an 8-GPU node.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
    --master-port 29511 bench.py --gpus 1 --steps 50 --warmup 10 --scenario flocking --envs 32768 \
    --n-agents 8 --cpu-steps 0 > gpurun_out/dist_c5.log 2>&1 || { echo "c5 failed"; tail -20 gpurun_out/dist_c5.log; exit 1; }
tail -1 gpurun_out/dist_c5.log
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
    --master-port 29512 bench.py --gpus 1 --steps 100 --warmup 10 --cpu-steps 0 \
    > gpurun_out/dist_c2.log 2>&1 || { echo "c2 failed"; tail -20 gpurun_out/dist_c2.log; exit 1; }
tail -1 gpurun_out/dist_c2.log
echo "dist done"
