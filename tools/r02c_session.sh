#!/bin/bash
# Round-2 GPU session c: RS calibration, GPU tests on the K1-lines build, default bench + its
# rocprofv3 kernel stats and FETCH/WRITE passes, configs[4] replica split rehearsal (2 ranks).
export TMPDIR=/tmp
tools/gpu_session.sh \
 "r02c_rs_ab:120:./tools/rs_ab" \
 "r02c_gpu_tests:600:python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
 "r02c_bench:200:python bench.py" \
 "r02c_kt:200:rocprofv3 --kernel-trace --stats -d gpurun_out/r02c_prof/kt -o kt --output-format csv -- python3 bench.py --no-cpu" \
 "r02c_fetch:200:rocprofv3 --pmc FETCH_SIZE -d gpurun_out/r02c_prof/fetch -o fetch --output-format csv -- python3 bench.py --no-cpu" \
 "r02c_write:200:rocprofv3 --pmc WRITE_SIZE -d gpurun_out/r02c_prof/write -o write --output-format csv -- python3 bench.py --no-cpu" \
 "r02c_cfg4:300:python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29513 bench.py --gpus 2 --dist-backend gloo --same-device --workload stream --total-objects 4000 --object-mib 1 --steps 2"
