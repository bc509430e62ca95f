#!/bin/bash
# Reproduce the committed profiles on a GPU box:  bash profiles/collect.sh <round-tag> [bench --config]
#   1. rocprofv3 --kernel-trace --stats of bench.py (same command line as the bench leg, short)
#   2. two SEPARATE --pmc passes (FETCH_SIZE and WRITE_SIZE do not fit one TCC pass on gfx950)
#   3. one SQ + GRBM pass: clock held under load (GRBM_GUI_ACTIVE), MFMA busy cycles, wave stall
#      breakdown (MI355X_MICROARCH.md §rocprofv3 PMC slots: 8 SQ + 2 GRBM per pass)
#   4. profiles/summarize.py -> profiles/<tag>_kernel_stats.md, profiles/pmc_traffic.json,
#      profiles/<tag>_sq_counters.md
set -euo pipefail
TAG=${1:-r01}
CFG=${2:-2}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=$ROOT/gpurun_out/prof_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
cd "$ROOT"
# CFG 2|3|4: bench.py --config CFG; 5 / 5x8: configs[4]'s per-GPU step (profiles/c5_step.py, bf16 / MXFP8)
if [ "$CFG" = 5 ] || [ "$CFG" = 5x8 ]; then
    X8=""; [ "$CFG" = 5x8 ] && X8="--fp8"
    PROG="profiles/c5_step.py $X8"
    ARGS="--steps 3 --warmup 1"; ARGS1="--steps 1 --warmup 1"
else
    PROG="bench.py --no-cpu-baseline --no-extra --config $CFG"
    ARGS="--steps 3 --warmup 1"; ARGS1="--steps 1 --warmup 0"
fi
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- \
    python3 $PROG $ARGS > "$OUT/trace.json" 2> "$OUT/trace.err"
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch" -o run -- \
    python3 $PROG $ARGS1 > "$OUT/fetch.json" 2> "$OUT/fetch.err"
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/write" -o run -- \
    python3 $PROG $ARGS1 > "$OUT/write.json" 2> "$OUT/write.err"
timeout -k 10 600 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
    SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE GRBM_COUNT \
    --output-format csv -d "$OUT/sq" -o run -- \
    python3 $PROG $ARGS1 > "$OUT/sq.json" 2> "$OUT/sq.err"
python3 profiles/summarize.py "$OUT" "$TAG"
