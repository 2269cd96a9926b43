#!/bin/bash
# Round evidence for the bench line: rocprofv3 kernel trace + stats of the driver's own command
# (`python bench.py`, default N = 1), then separate PMC passes (FETCH_SIZE, WRITE_SIZE; never with
# trace domains) over the headline workload alone, turned into per-launch HBM bytes.
# usage: bash tools/profile_bench.sh <outdir>
set -e
out=$1
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 900 rocprofv3 --kernel-trace --stats -d $out/kt -o kt --output-format csv -- python3 bench.py > $out/bench_kt.json
P="--no-extras --no-e2e --no-sweep --no-cpu --steps 2 --warmup 1"
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE -d $out/fetch -o fetch --output-format csv -- python3 bench.py $P > $out/bench_fetch.json
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE -d $out/write -o write --output-format csv -- python3 bench.py $P > $out/bench_write.json
python3 tools/pmc_traffic.py $(find $out/fetch -name 'fetch_counter_collection.csv') \
    $(find $out/write -name 'write_counter_collection.csv') $out/k1_traffic.json > /dev/null
