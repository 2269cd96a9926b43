#!/bin/bash
# Round-2 GPU session d: the nibble-table RS kernel -- parity tests, A/B vs round 1, bench line,
# rocprofv3 stats + FETCH/WRITE + LDS passes.
export TMPDIR=/tmp
tools/gpu_session.sh \
 "r02d_rs_tests:400:python -u -m pytest tests/test_rs_gpu.py tests/test_process_gpu.py -x -q --timeout 300 --timeout-method thread" \
 "r02d_rs_ab:120:./tools/rs_ab" \
 "r02d_rs_bench:200:python bench.py --workload rs" \
 "r02d_rs_prof:400:bash tools/profile_rs.sh r02"
tools/gpu_session.sh "r02d_bench_extras:400:python bench.py"
