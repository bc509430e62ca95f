#!/bin/bash
# A/B tuning: alternate bench runs across variant libraries (same box, interleaved rounds).
#   bash tests/ab_variants.sh "libcad_hip.so libcad_hip_bk32.so" 2
LIBS=${1:-libcad_hip.so}; ROUNDS=${2:-2}
mkdir -p gpurun_out
for r in $(seq 1 $ROUNDS); do
  for lib in $LIBS; do
    CAD_LIB=$lib timeout -k 10 240 python bench.py --steps 6 --warmup 2 --no-cpu-baseline \
      > gpurun_out/ab_${lib}_$r.json 2> gpurun_out/ab_${lib}_$r.err
    rc=$?; [ $rc -ge 124 ] && { echo "abort rc=$rc"; exit $rc; }
    python3 -c "import json,sys; d=json.load(open('gpurun_out/ab_${lib}_$r.json')); print('$lib', 'round', $r, d['value'], d['ms_per_step'])"
  done
done
