#!/bin/bash
# After the HIP-free fast path of dm_stream_write / dm_pstream_write.
export TMPDIR=/tmp
tools/gpu_session.sh \
 "r02t_stream_tests:400:python -u -m pytest tests/test_gpu_parity.py tests/test_process_gpu.py -x -q --timeout 200 --timeout-method thread -k 'stream'" \
 "r02t_host_tests:600:bash tests/cpp/run_host_tests.sh /tmp/deoss_hosttests" \
 "r02t_upload:300:python bench.py --workload upload --chunk 1048576 --object-gib 8 --steps 2 --warmup 1 --piece-kib 256"
