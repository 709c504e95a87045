#!/bin/bash
# PMC counter passes for one chain/shape (default: headline gaussian5, 16K RGB).
#   CH=blur:31 SHAPE=16384x2048x3 BAND=256 bash tools/gpu_prof.sh
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
CH=${CH:-gaussian5}
SHAPE=${SHAPE:-16384x16384x3}
BAND=${BAND:-0}
TAG=${TAG:-pmc}
i=0
for set in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE GRBM_COUNT" \
           "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR" \
           "SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_MISC SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM" \
           "FETCH_SIZE TCC_HIT_sum TCC_MISS_sum" "WRITE_SIZE TCC_EA0_RDREQ_sum"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $set -d gpurun_out/${TAG}$i -o run -- python tools/kbench.py --chains "$CH" --shape $SHAPE --bands $BAND --iters 6 --warmup 2 > gpurun_out/${TAG}$i.log 2>&1 || { echo "pmc set $i failed"; tail -5 gpurun_out/${TAG}$i.log; }
done
python tools/prof_summary.py gpurun_out/${TAG}*/run_results.db > gpurun_out/${TAG}_summary.txt 2>&1
grep -v "^_ZN6stripe3dev7k_synth" gpurun_out/${TAG}_summary.txt | head -80
