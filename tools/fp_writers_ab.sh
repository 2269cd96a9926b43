#!/bin/bash
# A/B of dm_full_processing's data-file writer count (DEOSS_FP_DATA_WRITERS) on an 8 GiB file.
set -e
mkdir -p gpurun_out/fp_writers
for rep in 1 2; do
  for w in 8 12 16; do
    DEOSS_FP_DATA_WRITERS=$w timeout -k 10 200 python bench.py --workload fullprocessing --object-gib 8 --steps 2 --warmup 1 --no-cpu \
      2>/dev/null | python -c "import sys,json; d=json.loads(sys.stdin.read()); print('writers $w rep $rep', d['ms_per_step'], d['step_ms'], d['host_io_floor']['ms'], d['parity']['bit_exact'])" | tee -a gpurun_out/fp_writers/summary.log
  done
done
