#!/bin/bash
# K1 at 4 KiB chunks (VERDICT r2 "what's weak" #5): the auto sweep read 1,411 GiB/s where the
# whole-line A/B read 1,506.  Same 8 GiB object, K1 forced: the main line at 4 KiB, a sweep that
# visits 4 KiB first, after 64 KiB and after 1 MiB (is it the order?), then separate rocprofv3
# passes: FETCH_SIZE, WRITE_SIZE, and SQ_INSTS_VALU + SQ_WAIT_INST_ANY + SQ_WAVE_CYCLES + GRBM_GUI_ACTIVE.
# usage: bash tools/k1_4k_probe.sh <outdir>
set -e
out=$1
mkdir -p $out
export TMPDIR=/tmp
A="--no-cpu --no-e2e --no-extras --chunk 4096 --leaf-kernel wide --steps 5 --warmup 1"
timeout -k 10 200 python bench.py $A --sweep --sweep-chunks 4096,65536,4096,1048576,4096,33554432,4096 > $out/bench_4k.json
P="--no-cpu --no-e2e --no-extras --no-sweep --chunk 4096 --leaf-kernel wide --steps 3 --warmup 1"
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $out/fetch -o fetch --output-format csv -- python3 bench.py $P > /dev/null
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $out/write -o write --output-format csv -- python3 bench.py $P > /dev/null
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_WAVES GRBM_GUI_ACTIVE -d $out/sq -o sq --output-format csv -- python3 bench.py $P > /dev/null
timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d $out/kt -o kt --output-format csv -- python3 bench.py $P > /dev/null
python3 tools/pmc_traffic.py $(find $out/fetch -name 'fetch_counter_collection.csv') \
    $(find $out/write -name 'write_counter_collection.csv') $out/traffic.json > $out/traffic.txt
