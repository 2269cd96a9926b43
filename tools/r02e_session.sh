#!/bin/bash
# Round-2 GPU session e: bench restructure (run_object), N=1 line with other_configs, and the
# 8-GPU extras path rehearsed with 2 gloo ranks on one GPU at reduced sizes.
export TMPDIR=/tmp
tools/gpu_session.sh \
 "r02e_bench:400:python bench.py" \
 "r02e_multi:400:python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29514 bench.py --gpus 2 --dist-backend gloo --same-device --object-gib 1 --steps 2 --multi-configs --cfg3-total-gib 4 --cfg4-objects 2000 --prefix-gib 1" \
 "r02e_smoke:120:python -c 'import __graft_entry__ as g; g.smoke()'"
