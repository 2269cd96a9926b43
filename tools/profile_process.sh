#!/bin/bash
# Profile the FullProcessing and proof benches (bench.py --workload process / proofs): kernel
# trace + stats, then separate PMC passes for HBM traffic (FETCH_SIZE, WRITE_SIZE).
# usage: tools/profile_process.sh <tag>
set -e
tag=${1:-r01}
out=gpurun_out/prof_proc_$tag
mkdir -p $out
export TMPDIR=/tmp
pa="--workload process --steps 2 --warmup 1 --no-cpu"
qa="--workload proofs --objects 1048576 --object-mib 0.00390625 --steps 3 --warmup 1"
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $out/pkt -o kt --output-format csv -- python3 bench.py $pa > $out/process_kt.json
timeout -k 10 240 rocprofv3 --pmc FETCH_SIZE -d $out/pfetch -o fetch --output-format csv -- python3 bench.py $pa > $out/process_fetch.json
timeout -k 10 240 rocprofv3 --pmc WRITE_SIZE -d $out/pwrite -o write --output-format csv -- python3 bench.py $pa > $out/process_write.json
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $out/qkt -o kt --output-format csv -- python3 bench.py $qa > $out/proofs_kt.json
timeout -k 10 240 rocprofv3 --pmc FETCH_SIZE -d $out/qfetch -o fetch --output-format csv -- python3 bench.py $qa > $out/proofs_fetch.json
