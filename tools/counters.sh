#!/bin/bash
# List gfx950 counters and collect SQ/GRBM counters for the wide leaf kernel (64 KiB chunks).
set -e
rocprofv3 -L > gpurun_out/counters_list.txt 2>&1 || true
rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVES SQ_INSTS_VALU SQ_BUSY_CYCLES -d gpurun_out/prof_sq1 -o sq1 --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu --no-e2e --chunk 65536 --object-gib 8 --no-sweep
rocprofv3 --pmc SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY -d gpurun_out/prof_sq2 -o sq2 --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu --no-e2e --chunk 65536 --object-gib 8 --no-sweep
