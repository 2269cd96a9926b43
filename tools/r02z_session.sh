#!/bin/bash
# Round-2 session z: zero-copy host paths -- their own tests first, then the full regression.
export TMPDIR=/tmp
tools/gpu_session.sh \
 "r02z_zc_tests:300:python -u -m pytest tests/test_zero_copy_gpu.py -x -v --timeout 120 --timeout-method thread" \
 "r02z_gpu_tests:700:python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
 "r02z_host_tests:600:bash tests/cpp/run_host_tests.sh /tmp/deoss_hosttests" \
 "r02z_smoke:120:python -c 'import __graft_entry__ as g; g.smoke()'" \
 "r02z_bench:400:python bench.py"
