#!/bin/bash
# Run a sequence of GPU steps on the gpurun box.  Each step has its own time limit; a step that
# crashes, aborts or times out (anything other than exit 0 = ok / 1 = test failures) ends the
# session so nothing else touches a possibly-wedged GPU.
#   tools/gpu_session.sh "<limit_s>|<name>|<command>" ...
mkdir -p gpurun_out
for spec in "$@"; do
  limit="${spec%%|*}"; rest="${spec#*|}"
  name="${rest%%|*}"; cmd="${rest#*|}"
  echo "[session] step $name (limit ${limit}s): $cmd"
  start=$(date +%s)
  timeout -k 10 "$limit" bash -c "$cmd" > "gpurun_out/${name}.log" 2>&1
  rc=$?
  echo "[session] step $name rc=$rc in $(( $(date +%s) - start ))s"
  tail -n 5 "gpurun_out/${name}.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then
    echo "[session] stopping after rc=$rc"
    exit $rc
  fi
done
exit 0
