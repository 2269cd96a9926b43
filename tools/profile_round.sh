#!/bin/bash
# Profile the bench command with rocprofv3: kernel trace + stats, then separate PMC passes for
# FETCH_SIZE and WRITE_SIZE (never combined with trace domains), then per-launch HBM traffic.
# usage: tools/profile_round.sh <round-tag> [extra bench args]
set -e
tag=${1:-r01}; shift || true
out=gpurun_out/prof_$tag
mkdir -p $out
args="--steps 2 --warmup 1 --no-cpu --sweep --sweep-modes $*"
rocprofv3 --kernel-trace --stats -d $out/kt -o kt --output-format csv -- python3 bench.py $args > $out/bench_kt.json
rocprofv3 --pmc FETCH_SIZE -d $out/fetch -o fetch --output-format csv -- python3 bench.py $args > $out/bench_fetch.json
rocprofv3 --pmc WRITE_SIZE -d $out/write -o write --output-format csv -- python3 bench.py $args > $out/bench_write.json
python3 tools/pmc_traffic.py $out/fetch/fetch_counter_collection.csv $out/write/write_counter_collection.csv $out/k1_traffic.json
