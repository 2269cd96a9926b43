#!/bin/bash
# Multi-rank rehearsals of the N > 1 bench path on the final tree (gloo ranks sharing cuda:0;
# printed as n_gpus 1 / ranks N / same_device): 2 and 8 ranks with the N = 8 extras at reduced size.
export TMPDIR=/tmp
tools/gpu_session.sh \
 "r02m_dist2:400:python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29514 bench.py --gpus 2 --dist-backend gloo --same-device --object-gib 1 --steps 2 --multi-configs --cfg3-total-gib 4 --cfg4-objects 2000 --prefix-gib 1" \
 "r02m_dist8:600:python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29515 bench.py --gpus 8 --dist-backend gloo --same-device --object-gib 0.25 --steps 2 --multi-configs --cfg3-total-gib 8 --cfg4-objects 8000 --prefix-gib 1"
