#!/bin/bash
# dm_full_processing: its GPU tests, the C++ host test (plain + ASan/UBSan), the file workload.
export TMPDIR=/tmp
tools/gpu_session.sh \
 "r02fp_tests:400:python -u -m pytest tests/test_process_gpu.py -x -v --timeout 200 --timeout-method thread -k full_processing" \
 "r02fp_host_tests:600:bash tests/cpp/run_host_tests.sh /tmp/deoss_hosttests" \
 "r02fp_bench8:400:python bench.py --workload fullprocessing --object-gib 8 --steps 2 --warmup 1"
