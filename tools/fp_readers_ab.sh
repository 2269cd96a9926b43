#!/bin/bash
# A/B of dm_full_processing's pread thread count (DEOSS_FP_READERS) on an 8 GiB file, phase trace on.
set -e
mkdir -p gpurun_out/fp_readers
for rep in 1 2; do
  for r in 8 12 16; do
    DEOSS_FP_TRACE=1 DEOSS_FP_READERS=$r timeout -k 10 200 python bench.py --workload fullprocessing --object-gib 8 --steps 2 --warmup 1 --no-cpu \
      > gpurun_out/fp_readers/r${r}_rep${rep}.log 2>&1
    python - gpurun_out/fp_readers/r${r}_rep${rep}.log $r $rep <<'PY' | tee -a gpurun_out/fp_readers/summary.log
import json, sys
lines = open(sys.argv[1]).read().splitlines()
d = json.loads([x for x in lines if x.startswith("{")][-1])
a = [float(x.split()[-2]) for x in lines if "A: reads" in x][-2:]
print("readers", sys.argv[2], "rep", sys.argv[3], d["ms_per_step"], d["step_ms"], "phaseA", a,
      "floor", d["host_io_floor"]["ms"], d["parity"]["bit_exact"])
PY
  done
done
