#!/bin/bash
# After sticky stream failures (dm_stream / dm_pstream), plus the bench with its new extra.
export TMPDIR=/tmp
tools/gpu_session.sh \
 "r02u2_tests:500:python -u -m pytest tests/test_process_gpu.py tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k 'stream or process'" \
 "r02u2_host_tests:600:bash tests/cpp/run_host_tests.sh /tmp/deoss_hosttests" \
 "r02u2_bench:600:python bench.py"
