#!/bin/bash
# The N = 8 rehearsal with the busiest processes sampled every 2 s (what else runs on the job's CPUs
# while the in-process leg measures its host feed).
mkdir -p gpurun_out
timeout -k 10 300 bash tools/rehearse_multi.sh 8 > gpurun_out/r05hf_e.log 2>&1 &
pid=$!
while kill -0 $pid 2>/dev/null; do
  sleep 2
  { date +%T; ps -eo pid,ppid,pcpu,stat,nlwp,args --sort=-pcpu | head -14 | cut -c1-160; echo ---; } >> gpurun_out/r05hf_ps.log
done
wait $pid
