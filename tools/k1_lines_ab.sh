#!/bin/bash
# A/B of K1's block loop: whole 128-B lines per iteration (DM_K1_LINES=1) vs one 64-B block
# (DM_K1_LINES=0).  Per variant: the bench at 64 KiB chunks + a 4 KiB sweep point with K1 forced
# (HIP-event rates), then separate rocprofv3 FETCH_SIZE / WRITE_SIZE passes -> per-launch traffic.
# usage: bash tools/k1_lines_ab.sh <outdir> variant...   (variant = build_variants/<name>.so)
set -e
out=$1; shift
mkdir -p $out
export TMPDIR=/tmp
args=${ARGS:-"--no-cpu --chunk 65536 --leaf-kernel wide --sweep --sweep-chunks 4096,65536 --sweep-modes --steps 3 --warmup 1"}
for v in "$@"; do
  lib=$PWD/build_variants/$v.so
  DEOSS_MERKLE_LIB=$lib timeout -k 10 120 python bench.py $args > $out/$v.bench.json
  DEOSS_MERKLE_LIB=$lib timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE -d $out/$v.fetch -o fetch --output-format csv -- python3 bench.py $args > /dev/null
  DEOSS_MERKLE_LIB=$lib timeout -k 10 120 rocprofv3 --pmc WRITE_SIZE -d $out/$v.write -o write --output-format csv -- python3 bench.py $args > /dev/null
  python3 tools/pmc_traffic.py $(find $out/$v.fetch -name 'fetch_counter_collection.csv') \
      $(find $out/$v.write -name 'write_counter_collection.csv') $out/$v.traffic.json > /dev/null
  python3 - $out/$v.bench.json $out/$v.traffic.json <<'PY'
import json, sys
b = json.load(open(sys.argv[1])); t = json.load(open(sys.argv[2]))["by_kernel_grid"]
print("main", b["value"], "GiB/s", "k1", b["roofline"]["k1_avg_ms"], "ms")
for e in b["sweep"]:
    print("sweep", e["chunk"], e["leaf_kernel"], e["gibs"], "GiB/s", e["k1_gbs"], "GB/s")
alg = {}
for k, v in sorted(t.items()):
    print("traffic", k, v["hbm_bytes_per_launch"], "x%.4f" % (v["hbm_bytes_per_launch"] / 8589934592))
PY
done
