#!/bin/bash
# 8 idle processes holding a HIP context on GPU 0 while the in-process leg runs alone
pids=()
for i in 0 1 2 3 4 5 6 7; do
  python -c "import torch,time; torch.zeros(1,device='cuda'); time.sleep(90)" &
  pids+=($!)
done
sleep 20
timeout -k 10 200 python bench.py --workload inprocess --inproc-gib 16 --inproc-devices 8
rc=$?
kill "${pids[@]}" 2>/dev/null
wait
exit $rc
