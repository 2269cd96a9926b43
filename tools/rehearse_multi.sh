#!/bin/bash
# Rehearse the driver's N > 1 bench path on ONE GPU: N gloo ranks all on cuda:0 (reported as
# "same_device"), the weak-scaling line plus the 8-GPU extras (configs[3] / configs[4]) at reduced
# sizes and the in-process leg (virtual devices standing in for the GPUs), every parity leg on.
# Not a multi-GPU measurement: it exercises the code path the driver's 8-GPU run takes.  bench.py
# starts the ranks itself (no WORLD_SIZE: child torch.distributed.run), as a bare `--gpus N` does.
# usage: bash tools/rehearse_multi.sh <ranks>
set -e
n=${1:-8}
export TMPDIR=/tmp
python bench.py --gpus $n --dist-backend gloo --same-device --object-gib 0.25 --steps 2 --multi-configs \
  --cfg3-total-gib 8 --cfg4-objects 8000 --prefix-gib 1 --in-process --inproc-gib 16
