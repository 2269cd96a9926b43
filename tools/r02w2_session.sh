#!/bin/bash
# dm_full_processing with data files copied from the file during the leaf pass (copy_file_range).
export TMPDIR=/tmp
tools/gpu_session.sh \
 "r02w2_tests:400:python -u -m pytest tests/test_process_gpu.py -x -q --timeout 200 --timeout-method thread" \
 "r02w2_host_tests:600:bash tests/cpp/run_host_tests.sh /tmp/deoss_hosttests" \
 "r02w2_fp8:400:python bench.py --workload fullprocessing --object-gib 8 --steps 2 --warmup 1" \
 "r02w2_fp2:300:python bench.py --workload fullprocessing --object-gib 2 --steps 3 --warmup 1"
