#!/bin/bash
# Round-2 GPU session l: full regression on the current build.
export TMPDIR=/tmp
tools/gpu_session.sh \
 "r02l_gpu_tests:700:python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
 "r02l_host_tests:600:bash tests/cpp/run_host_tests.sh /tmp/deoss_hosttests" \
 "r02l_smoke:120:python -c 'import __graft_entry__ as g; g.smoke()'" \
 "r02l_bench:400:python bench.py"
