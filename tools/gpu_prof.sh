#!/bin/bash
# Band sweep + PMC counter passes for the headline kernel (gaussian5, 16K RGB).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
CH=${CH:-gaussian5}
timeout -k 10 300 python tools/kbench.py --chains "$CH" --bands 16,24,32,48,64,106,160,256 --iters 30 > gpurun_out/bands.log 2>&1 || exit 1
cat gpurun_out/bands.log
i=0
for set in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE GRBM_COUNT" \
           "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR" \
           "FETCH_SIZE TCC_HIT_sum TCC_MISS_sum" "WRITE_SIZE TCC_EA0_RDREQ_sum"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $set -d gpurun_out/pmc$i -o run -- python tools/kbench.py --chains "$CH" --iters 6 --warmup 2 > gpurun_out/pmc$i.log 2>&1 || { echo "pmc set $i failed"; tail -5 gpurun_out/pmc$i.log; }
done
python tools/prof_summary.py gpurun_out/pmc*/run_results.db > gpurun_out/pmc_summary.txt 2>&1
cat gpurun_out/pmc_summary.txt | grep -v "^_ZN6stripe3dev7k_synth" | head -80
