#!/bin/bash
# Profile one filter chain on one MI355X with rocprofv3 (SURVEY §5 "tracing /
# profiling"): a kernel trace with per-kernel stats, then counter passes (each
# --pmc pass in its own run, never combined with the system/runtime traces).
#
#   scripts/profile.sh [CHAIN] [WxHxC] [OUTDIR]
#   scripts/profile.sh gaussian5 16384x16384x3 gpurun_out/prof_g5
#
# Counter notes (gfx950): FETCH_SIZE reads half the bytes on this part
# (MI355X_MICROARCH.md); SQ_* cycle counters count quad-cycles except
# SQ_VALU_MFMA_BUSY_CYCLES; sums are over hardware instances (tools/prof_summary.py).
set -o pipefail
CHAIN=${1:-gaussian5}
SHAPE=${2:-16384x16384x3}
OUT=${3:-gpurun_out/profile}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
case "$OUT" in /*) ;; *) OUT="$ROOT/$OUT" ;; esac
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
KB=(python3 "$ROOT/tools/kbench.py" --chains "$CHAIN" --shape "$SHAPE")
[ -n "$BANDS" ] && KB+=(--bands "$BANDS")  # e.g. BANDS=8: a fixed band height (the tuner's pick)
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run -- "${KB[@]}" --iters 20 > "$OUT/trace.log" 2>&1 || { tail -20 "$OUT/trace.log"; exit 1; }
i=0
for set in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE" \
           "SQ_INSTS_VALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE" \
           "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $set -d "$OUT/pmc$i" -o run -- "${KB[@]}" --iters 4 --warmup 1 > "$OUT/pmc$i.log" 2>&1 || { echo "counter set $i failed (see $OUT/pmc$i.log)"; }
done
python3 "$ROOT/tools/prof_summary.py" "$OUT"/trace/run_results.db "$OUT"/pmc*/run_results.db > "$OUT/summary.txt" 2>&1
grep -v "k_synth" "$OUT/summary.txt" | head -60
