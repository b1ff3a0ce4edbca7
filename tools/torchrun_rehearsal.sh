#!/bin/bash
# torchrun path of bench.py with 2 ranks sharing the box's one GPU (QPP_SHARE_DEVICE=1): checks the launch,
# sharding, barrier and max-over-ranks plumbing the driver's N>1 runs use.  Not a scaling measurement.
set -o pipefail
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp
mkdir -p gpurun_out/tr
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 1 --steps 5 --warmup 2 > gpurun_out/tr/n1.json 2> gpurun_out/tr/n1.err || { tail -20 gpurun_out/tr/n1.err; exit 1; }
cat gpurun_out/tr/n1.json
QPP_SHARE_DEVICE=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 2 --steps 5 --warmup 2 --no-cpu > gpurun_out/tr/n2.json 2> gpurun_out/tr/n2.err || { tail -20 gpurun_out/tr/n2.err; exit 1; }
cat gpurun_out/tr/n2.json
# BASELINE configs[4] shape on 2 ranks (strong split of a fixed total, 4096 rotating keys, end to end)
QPP_SHARE_DEVICE=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29513 bench.py --gpus 2 --mode e2e --keys 4096 --rotate --total-packets 2097152 --steps 2 --warmup 1 > gpurun_out/tr/c5.json 2> gpurun_out/tr/c5.err || { tail -20 gpurun_out/tr/c5.err; exit 1; }
cat gpurun_out/tr/c5.json
