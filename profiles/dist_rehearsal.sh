#!/bin/bash
# Rehearse the driver's multi-GPU launch on a one-GPU box (repo root, under gpurun):
# torchrun with 1 rank over RCCL, then 2 ranks sharing cuda:0 over gloo.
set -e
OUT=gpurun_out/dist
mkdir -p $OUT
timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29511 \
  bench.py --gpus 1 --steps 10 --warmup 20 --no-cpu-baseline --no-cache-window > $OUT/n1_rccl.json 2> $OUT/n1_rccl.err
timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29512 \
  bench.py --gpus 2 --steps 10 --warmup 20 --no-cpu-baseline --no-cache-window --dist-backend gloo > $OUT/n2_gloo.json 2> $OUT/n2_gloo.err
