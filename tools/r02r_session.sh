#!/bin/bash
# Round-2 regression after dm_full_processing / dm_pstream: every GPU test, host tests, smoke,
# the default bench line (with its other_configs), and rocprofv3 kernel stats of the headline.
export TMPDIR=/tmp
tools/gpu_session.sh \
 "r02r_gpu_tests:800:python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
 "r02r_smoke:120:python -c 'import __graft_entry__ as g; g.smoke()'" \
 "r02r_bench:600:python bench.py" \
 "r02r_prof:300:rocprofv3 --kernel-trace --stats -d gpurun_out/r02r_prof -o kt --output-format csv -- python3 bench.py --no-extras --steps 5 --warmup 1"
