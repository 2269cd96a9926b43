#!/bin/bash
# Round-2 GPU session g: pipelined host batches -- parity tests, configs[4] share before/after.
export TMPDIR=/tmp
tools/gpu_session.sh \
 "r02g_tests:400:python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k 'batch or golden'" \
 "r02g_stream:200:python bench.py --workload stream --objects 12500 --object-mib 1 --steps 3" \
 "r02g_stream_base:200:DEOSS_MERKLE_LIB=build_variants/k1_lines.so python bench.py --workload stream --objects 12500 --object-mib 1 --steps 3"
