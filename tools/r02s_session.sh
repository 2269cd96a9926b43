#!/bin/bash
# After lazily pinned pstream slots / sync on failed calls / the C++ process mirror.
export TMPDIR=/tmp
tools/gpu_session.sh \
 "r02s_process_tests:500:python -u -m pytest tests/test_process_gpu.py -x -q --timeout 200 --timeout-method thread" \
 "r02s_host_tests:600:bash tests/cpp/run_host_tests.sh /tmp/deoss_hosttests"
