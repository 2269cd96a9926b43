#!/bin/bash
# Profile the Reed-Solomon bench (bench.py --workload rs): kernel trace + stats, then separate PMC
# passes (HBM traffic: FETCH_SIZE, WRITE_SIZE; LDS: bank conflicts; VALU activity).
# usage: tools/profile_rs.sh <tag>
set -e
tag=${1:-r01}
out=gpurun_out/prof_rs_$tag
mkdir -p $out
args="--workload rs --steps 2 --warmup 1 --no-cpu"
rocprofv3 --kernel-trace --stats -d $out/kt -o kt --output-format csv -- python3 bench.py $args > $out/bench_kt.json
rocprofv3 --pmc FETCH_SIZE -d $out/fetch -o fetch --output-format csv -- python3 bench.py $args > $out/bench_fetch.json
rocprofv3 --pmc WRITE_SIZE -d $out/write -o write --output-format csv -- python3 bench.py $args > $out/bench_write.json
rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS GRBM_GUI_ACTIVE -d $out/lds -o lds --output-format csv -- python3 bench.py $args > $out/bench_lds.json
rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES -d $out/valu -o valu --output-format csv -- python3 bench.py $args > $out/bench_valu.json
