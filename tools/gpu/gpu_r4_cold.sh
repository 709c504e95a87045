mkdir -p gpurun_out/r4
for h in 256 512 1024 2048 4096 8192; do
  timeout -k 10 100 python tools/coldbench.py --shape 16384x${h}x3 --bands 8,12,16,24 --caps=-1,2 --nt 1 > gpurun_out/r4/cold_h${h}.txt 2>&1 || exit 1
done
timeout -k 10 100 python tools/coldbench.py --frames 1 --bands 8,12,16 --caps=-1,0,2 --nt 0,1 > gpurun_out/r4/warm_f1.txt 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/r4/prof_cold -o cold -- python3 tools/coldbench.py --bands 12 --caps=-1 --nt 1 --steps 40 > gpurun_out/r4/prof_cold.txt 2>&1 || exit 1
timeout -k 10 200 python bench.py --steps 20 --warmup 5 > gpurun_out/r4/bench_n1.json 2> gpurun_out/r4/bench_n1.err || exit 1
timeout -k 10 200 python bench.py --steps 20 --warmup 5 --height 2048 > gpurun_out/r4/bench_stripe.json 2> gpurun_out/r4/bench_stripe.err || exit 1
