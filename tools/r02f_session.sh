#!/bin/bash
# Round-2 GPU session f: new tests (special files, segment files), 8 gloo ranks on one GPU through
# the whole N = 8 bench path (weak line + configs[3]/[4] extras at reduced sizes).
export TMPDIR=/tmp
tools/gpu_session.sh \
 "r02f_tests:400:python -u -m pytest tests/test_gpu_parity.py tests/test_process_gpu.py -x -q --timeout 300 --timeout-method thread -k 'files or special or go_errors or last_error or process'" \
 "r02f_dist8:600:python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29515 bench.py --gpus 8 --dist-backend gloo --same-device --object-gib 0.25 --steps 2 --multi-configs --cfg3-total-gib 8 --cfg4-objects 8000 --prefix-gib 1"
