#!/bin/bash
# A/B of the K1Q step: shipped (8 VALU, 4-deep chain: alignbit -> xor_dpp -> xor_dpp -> add3) vs
# DM_QS_DEEP3=1 (9 VALU, 3-deep chain: three same-lane alignbits -> xor3 -> add3).  Interleaved
# repeats of the headline (8 GiB as 256 x 32 MiB, K1Q forced), the compact launch (1 MiB chunks)
# and the configs[2] batch; then the K1Q parity tests against the variant library.
# usage: bash tools/deep3_ab.sh   (abv/{base,deep3}.so; abv/ travels to the GPU box, build_variants/ does not)
set -e
out=gpurun_out/deep3
mkdir -p $out
one() { # lib args...
  local lib=$1; shift
  DEOSS_MERKLE_LIB=$PWD/abv/$lib.so timeout -k 10 150 python bench.py --no-cpu --steps 3 --warmup 1 "$@" \
    2>>$out/stderr.log | python -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d.get("parity",{}).get("bit_exact"))'
}
for rep in 1 2; do
  for v in base deep3; do
    echo "$v rep$rep 32MiB: $(one $v --chunk 33554432 --leaf-kernel quad)" | tee -a $out/summary.log
    echo "$v rep$rep 1MiB: $(one $v --chunk 1048576 --leaf-kernel quad)" | tee -a $out/summary.log
    echo "$v rep$rep batch4096x4MiB: $(one $v --workload batch --objects 4096 --object-mib 4)" | tee -a $out/summary.log
  done
done
DEOSS_MERKLE_LIB=$PWD/abv/deep3.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q \
  --timeout 120 --timeout-method thread -k "quad or golden or full_size" 2>&1 | tail -3 | tee -a $out/summary.log
