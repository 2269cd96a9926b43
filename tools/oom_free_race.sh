#!/bin/bash
# Build tools/oom_free_race{,.so} (here, on the CPU) -- run on the GPU box with tools/oom_free_race.py.
set -euo pipefail
cd "$(dirname "$0")"
hipcc --offload-arch=gfx950 -O2 -DOOM_RACE_MAIN -o oom_free_race oom_free_race.hip -lpthread
hipcc --offload-arch=gfx950 -O2 -fPIC -shared -o liboom_free_race.so oom_free_race.hip -lpthread
