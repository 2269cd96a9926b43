# usage: bash tools/ab_builds.sh base exp ...  (each name = build_variants/<name>.so, built with hipcc from a patched tree)
# A/B library builds (build_variants/*.so) on the K1Q wide (32 MiB chunks) and compact (1 MiB)
# launches and on table-mode batches (4096 x 4 MiB: wide, 6144 x 2 MiB: compact)
set -e
run() { # lib chunk
  echo "$1 chunk $2: $(DEOSS_MERKLE_LIB=build_variants/$1.so timeout -k 10 120 python bench.py --no-cpu --chunk $2 --leaf-kernel quad --steps 3 --warmup 1 2>/dev/null | python -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"])')"
}
batch() { # lib objects mib
  echo "$1 batch $2 x $3 MiB: $(DEOSS_MERKLE_LIB=build_variants/$1.so timeout -k 10 120 python bench.py --workload batch --objects $2 --object-mib $3 --steps 3 --warmup 1 2>/dev/null | python -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["parity"]["bit_exact"])')"
}
for v in "$@"; do run $v 33554432; run $v 1048576; run $v 2097152; batch $v 4096 4; batch $v 6144 2; done
