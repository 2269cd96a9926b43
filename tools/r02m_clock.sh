#!/bin/bash
# Round-2 session m: effective shader clock and issue counters of the headline K1Q launch
# (GRBM_GUI_ACTIVE / 8 XCDs / kernel duration; SQ wave-cycle counters), one --pmc pass each.
export TMPDIR=/tmp
B="python3 bench.py --steps 2 --warmup 1 --no-cpu --no-extras"
tools/gpu_session.sh \
 "r02m_pmc1:120:rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE SQ_WAVES SQ_INSTS_VALU SQ_BUSY_CYCLES -d gpurun_out/r02m_pmc1 -o pmc1 --output-format csv -- $B" \
 "r02m_pmc2:120:rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY -d gpurun_out/r02m_pmc2 -o pmc2 --output-format csv -- $B" \
 "r02m_pmc3:120:rocprofv3 --kernel-trace --pmc SQ_INST_CYCLES_VALU SQ_ACTIVE_INST_ANY SQ_INSTS_SALU SQ_INSTS_LDS -d gpurun_out/r02m_pmc3 -o pmc3 --output-format csv -- $B"
