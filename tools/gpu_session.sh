#!/bin/bash
# Run GPU steps in order; stop at the first fault-like exit (timeout/abort/segfault/kill).
# usage: tools/gpu_session.sh "<name>:<timeout_s>:<command>" ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
rc_all=0
for spec in "$@"; do
  name="${spec%%:*}"; rest="${spec#*:}"; tmo="${rest%%:*}"; cmd="${rest#*:}"
  echo "=== [$name] (limit ${tmo}s): $cmd"
  start=$(date +%s)
  timeout -k 10 "$tmo" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "=== [$name] exit $rc after $(( $(date +%s) - start ))s"
  tail -n 25 "gpurun_out/$name.log"
  if [ $rc -ne 0 ]; then rc_all=$rc; fi
  case $rc in
    124|134|137|139|143) echo "=== fault-like exit $rc: stopping"; exit $rc;;
  esac
done
exit $rc_all
