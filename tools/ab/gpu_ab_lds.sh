set -o pipefail
CH="gaussian5;sobel;gaussian3;box5;gaussian7" bash tools/gpu_ab.sh || exit 1
timeout -k 10 300 python -m pytest tests/test_gpu_kernels.py -x -q -k "stencil_exact or chains" -p no:cacheprovider 2>&1 | tail -2
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --pmc SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE -d $GRAFT_REPO_ROOT/gpurun_out/pmc_lds -o run -- python3 $GRAFT_REPO_ROOT/tools/kbench.py --chains gaussian5 --iters 4 --warmup 1 > $GRAFT_REPO_ROOT/gpurun_out/pmc_lds.log 2>&1
cd $GRAFT_REPO_ROOT && python tools/prof_summary.py gpurun_out/pmc_lds/run_results.db | grep -A6 "k_sep" | tail -6
