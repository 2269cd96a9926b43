#!/bin/bash
# Round-2 GPU session h: full regression on the current build.
export TMPDIR=/tmp
tools/gpu_session.sh \
 "r02h_gpu_tests:700:python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
 "r02h_host_tests:600:bash tests/cpp/run_host_tests.sh /tmp/deoss_hosttests" \
 "r02h_smoke:120:python -c 'import __graft_entry__ as g; g.smoke()'" \
 "r02h_bench:400:python bench.py"
