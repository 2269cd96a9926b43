#!/bin/bash
# Full-size per-rank work of each leg of the N = 8 bench line, timed on ONE MI355X (VERDICT r5
# item 1: the first real 8-GPU line must fit the driver's time limit).  Each step is a fresh
# `python bench.py` process doing what one rank (or, for the in-process leg, rank 0's child)
# does in that leg at full size, so every wall time below also pays a torch import and a context
# creation the real leg does not -- an upper bound per leg.  DESIGN.md §8 sums them against
# bench.py's --deadline-s default.
#   headline_parity_64g  rank 0's single-GPU root of the whole 64 GiB weak object (the N = 8
#                        headline's parity leg; the 8 GiB per-rank timed steps are the N = 1 line)
#   strong_4k_8g         configs[1]'s 8 GiB at 4 KiB chunks on one GPU (the strong_scaling_4KiB
#                        leg's single-GPU reference; each rank's share is 1/8 of it)
#   cfg3_share_128g      configs[3]'s per-rank share: 128 GiB, 4,096 leaves of 32 MiB, 1 + 3 steps
#   cfg4_share_12500     configs[4]'s per-rank share: 12,500 x 1 MiB pinned host objects, 1 + 2
#                        steps, every root checked on the CPU
#   inprocess_8virt_64g  the in-process leg: 64 GiB pinned object over 8 virtual devices, batch,
#                        concurrent calls, host feed
# usage (on the GPU box): tools/n8_leg_times.sh  -> gpurun_out/n8_legs/{<leg>.json,<leg>.err,times.jsonl}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
out=gpurun_out/n8_legs
mkdir -p "$out"
: > "$out/times.jsonl"

leg() {   # leg <name> <limit_s> <bench args...>
    local name=$1 limit=$2
    shift 2
    local t0 t1 rc
    echo "[n8_leg_times] $(date +%T) $name: bench.py $*"
    t0=$(date +%s.%N)
    timeout -k 10 "$limit" python -u bench.py "$@" > "$out/$name.json" 2> "$out/$name.err"
    rc=$?
    t1=$(date +%s.%N)
    python3 -c "import json,sys; print(json.dumps({'leg': sys.argv[1], 'rc': int(sys.argv[2]), 'wall_s': round(float(sys.argv[4]) - float(sys.argv[3]), 1), 'args': sys.argv[5:]}))" \
        "$name" "$rc" "$t0" "$t1" "$@" >> "$out/times.jsonl"
    tail -n 1 "$out/times.jsonl"
    return $rc
}

leg headline_parity_64g 240 --total-gib 64 --steps 3 --warmup 1 --no-extras --no-cpu &&
leg strong_4k_8g 240 --total-gib 8 --chunk 4096 --steps 20 --warmup 3 --no-extras --no-cpu &&
leg cfg3_share_128g 300 --total-gib 128 --steps 3 --warmup 1 --no-extras --no-cpu &&
leg cfg4_share_12500 300 --workload stream --objects 12500 --object-mib 1 --steps 2 --warmup 1 &&
leg inprocess_8virt_64g 480 --workload inprocess --same-device --inproc-devices 8 --inproc-gib 64
