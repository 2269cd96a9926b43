#!/bin/bash
# dm_pstream: its GPU tests and the handler-flow workload (C++ host test: r02ps_host_tests.log).
export TMPDIR=/tmp
tools/gpu_session.sh \
 "r02ps_tests:400:python -u -m pytest tests/test_process_gpu.py -x -v --timeout 200 --timeout-method thread -k 'processing_stream or full_processing'" \
 "r02ps_bench:400:python bench.py --workload process_upload --object-gib 8 --steps 2 --warmup 1"
