tools/gpu_session.sh \
 "r02b_gpu_tests:600:python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
 "r02b_host_tests:600:bash tests/cpp/run_host_tests.sh /tmp/deoss_hosttests" \
 "r02b_bench:200:python bench.py" \
 "r02b_files:300:python bench.py --workload files --steps 3 --warmup 1" \
 "r02b_plumbing:120:python bench.py --workload plumbing" \
 "r02b_dist2:300:python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --dist-backend gloo --same-device --object-gib 1 --prefix-gib 0.5 --steps 2" \
 "r02b_dist2t:300:python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 2 --dist-backend gloo --same-device --total-gib 4 --prefix-gib 1 --steps 2"
