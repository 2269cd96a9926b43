#!/bin/bash
# Round-2 final regression: every GPU test, host tests (plain + ASan/UBSan), smoke, the default
# bench line with its other_configs, rocprofv3 kernel stats of the headline.
export TMPDIR=/tmp
tools/gpu_session.sh \
 "r02z2_gpu_tests:800:python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
 "r02z2_host_tests:600:bash tests/cpp/run_host_tests.sh /tmp/deoss_hosttests" \
 "r02z2_smoke:120:python -c 'import __graft_entry__ as g; g.smoke()'" \
 "r02z2_bench:600:python bench.py" \
 "r02z2_prof:300:rocprofv3 --kernel-trace --stats -d gpurun_out/r02z2_prof -o kt --output-format csv -- python3 bench.py --no-extras --steps 5 --warmup 1"
