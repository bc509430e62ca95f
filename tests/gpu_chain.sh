#!/bin/bash
# Run GPU steps in order; each step "name|timeout|command". Ordinary failures (exit 1..2) are
# recorded and the chain continues; a fault/abort/timeout (>=124) stops the chain.
mkdir -p gpurun_out
while IFS= read -r line; do
  [ -z "$line" ] && continue
  name=${line%%|*}; rest=${line#*|}; to=${rest%%|*}; cmd=${rest#*|}
  timeout -k 10 "$to" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "step $name exit=$rc"; tail -3 "gpurun_out/$name.log"
  if [ $rc -ge 124 ]; then echo "stopping chain after $name (rc=$rc)"; exit $rc; fi
done
