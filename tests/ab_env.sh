#!/bin/bash
# A/B tuning over environment settings (same box, interleaved rounds):
#   bash tests/ab_env.sh ROUNDS "NAME1:VAR=1,VAR2=2" "NAME2:" ...
# prints the bench value per arm per round and the top kernels of the last round of each arm.
ROUNDS=${1:-2}; shift
mkdir -p gpurun_out
for r in $(seq 1 $ROUNDS); do
  for arm in "$@"; do
    name=${arm%%:*}; vars=${arm#*:}
    env $(echo "$vars" | tr ',' ' ') timeout -k 10 240 python bench.py --steps 6 --warmup 2 --no-cpu-baseline \
      > gpurun_out/ab_${name}_$r.json 2> gpurun_out/ab_${name}_$r.err
    rc=$?; [ $rc -ge 124 ] && { echo "abort rc=$rc"; exit $rc; }
    python3 -c "import json; d=json.load(open('gpurun_out/ab_${name}_$r.json')); print('$name', 'round', $r, d['value'], d['ms_per_step'])"
  done
done
