#!/bin/bash
# Memory-side traffic (rocprofv3 PMC) of one step of every extra workload bench.py's N = 1 line
# reports under other_configs, at the sizes driver_extras() runs them: for each, two separate
# passes (FETCH_SIZE, WRITE_SIZE: they do not fit one pass, MI355X_MICROARCH.md "PMC slots") over
# `bench.py --workload ... --warmup 0 --steps K --no-cpu` for K = 1 and 2; tools/pmc_extras.py
# takes the difference per kernel (the marginal, warm step: setup and the parity check cancel)
# into profiles/extras_traffic.json (read by bench.py at run time, so it lives outside the
# gpurun-ignored round directories).
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
  for k in 1 2; do
    a="${EXTRAS[$n]} --warmup 0 --steps $k --no-cpu"
    o="$out/$n/s$k"
    mkdir -p "$o"
    for c in FETCH_SIZE WRITE_SIZE; do
      echo "=== $n steps $k $c: bench.py $a"
      timeout -s KILL 300 rocprofv3 --pmc $c -d "$o/$c" -o pmc --output-format csv -- python3 bench.py $a \
        > "$o/$c.json" 2> "$o/$c.err"
      rc=$?
      echo "=== $n steps $k $c exit $rc"
      if [ $rc -ne 0 ]; then tail -5 "$o/$c.err"; exit $rc; fi
    done
  done
  echo "${EXTRAS[$n]} --warmup 0 --steps {1,2} --no-cpu" > "$out/$n/args.txt"
done
# gpurun merges only gpurun_out/ back: write the summary there too, then copy it to profiles/
# locally (or rerun pmc_extras.py on the merged CSVs, which gives the same file)
python3 tools/pmc_extras.py "$out" "$out/extras_traffic.json" "$tag" && cp "$out/extras_traffic.json" profiles/extras_traffic.json
