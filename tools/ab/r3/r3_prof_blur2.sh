#!/bin/bash
# blur:31 16K RGB counter passes (one rocprofv3 run per pass, counters only)
set -o pipefail
ROOT=$(pwd); OUT=$ROOT/gpurun_out/r3prof_blur2; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
KB=(python3 "$ROOT/tools/kbench.py" --chains 'blur:31|' --shape 16384x16384x3)
timeout -k 10 120 rocprofv3 -L > $OUT/avail.txt 2>&1 || true
grep -o "SQ_[A-Z_0-9]*" $OUT/avail.txt | sort -u > $OUT/sq_avail.txt || true
i=0
for set in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE" \
           "SQ_INSTS_VALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE" \
           "SQ_VALU_MFMA_COEXEC_CYCLES SQ_INSTS_MFMA SQ_INSTS_SALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_INSTS_VMEM_RD"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $set -d "$OUT/pmc$i" -o run -- "${KB[@]}" --iters 4 --warmup 1 > "$OUT/pmc$i.log" 2>&1 || { echo "counter set $i failed"; tail -3 $OUT/pmc$i.log; }
done
python3 "$ROOT/tools/prof_summary.py" "$OUT"/pmc*/run_results.db > "$OUT/summary.txt" 2>&1
grep -A30 "k_blur_pl" "$OUT/summary.txt" | grep -v "^_ZN6stripe3dev7k_synth\|fillBuffer\|copyBuffer" | head -60
