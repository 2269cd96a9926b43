#!/bin/bash
# Memory-side traffic (rocprofv3 PMC) of one step of every extra workload bench.py's N = 1 line
# reports under other_configs, at the sizes driver_extras() runs them: for each, two separate
# passes (FETCH_SIZE, WRITE_SIZE: they do not fit one pass, MI355X_MICROARCH.md "PMC slots") over
# `bench.py --workload ... --warmup 0 --steps 1 --no-cpu`, then tools/pmc_extras.py sums every
# kernel the step launched (not the synthetic-data fill) into profiles/extras_traffic.json (read by
# bench.py at run time, so it lives outside the gpurun-ignored round directories).
# usage: bash tools/profile_extras.sh <tag> [name ...]   (names: see EXTRAS below; default all)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
tag=${1:-r04}
shift
out=gpurun_out/${tag}_pmc
mkdir -p "$out"
declare -A EXTRAS=(
  [configs0]="--workload plumbing"
  [configs2]="--workload batch --objects 4096 --object-mib 4"
  [configs4]="--workload stream --objects 12500 --object-mib 1"
  [files]="--workload files --objects 256 --object-mib 32"
  [upload]="--workload upload --chunk 1048576 --object-gib 8"
  [process]="--workload process --object-gib 8"
  [rs]="--workload rs --object-gib 8"
  [fullprocessing]="--workload fullprocessing --object-gib 2 --no-aux"
  [process_upload]="--workload process_upload --object-gib 2 --piece-kib 1024 --no-aux"
)
names=("$@")
[ ${#names[@]} -eq 0 ] && names=(configs0 configs2 configs4 files upload process rs fullprocessing process_upload)
for n in "${names[@]}"; do
  a="${EXTRAS[$n]} --warmup 0 --steps 1 --no-cpu"
  mkdir -p "$out/$n"
  for c in FETCH_SIZE WRITE_SIZE; do
    echo "=== $n $c: bench.py $a"
    timeout -s KILL 300 rocprofv3 --pmc $c -d "$out/$n/$c" -o pmc --output-format csv -- python3 bench.py $a \
      > "$out/$n/$c.json" 2> "$out/$n/$c.err"
    rc=$?
    echo "=== $n $c exit $rc"
    if [ $rc -ne 0 ]; then tail -5 "$out/$n/$c.err"; exit $rc; fi
  done
  echo "$a" > "$out/$n/args.txt"
done
python3 tools/pmc_extras.py "$out" profiles/extras_traffic.json "$tag"
