mkdir -p gpurun_out/r4
for st in 1 2; do for sti in 1 0; do
timeout -k 10 100 python tools/coldbench.py --bands 8,12,16,24 --caps=-1,2,3 --nt 1 --streams $st --stage-timing $sti > gpurun_out/r4/cold_s${st}_t${sti}.txt 2>&1 || exit 1
done; done
timeout -k 10 100 python tools/coldbench.py --shape 8192x2048x1 --chain sobel --bands 4,8,12 --caps=-1,2 --nt 0,1 --streams 1 --stage-timing 0 > gpurun_out/r4/sobel_s1.txt 2>&1 || exit 1
timeout -k 10 100 python tools/coldbench.py --shape 8192x2048x1 --chain sobel --bands 4,8,12 --caps=-1,2 --nt 0,1 --streams 2 --stage-timing 0 > gpurun_out/r4/sobel_s2.txt 2>&1 || exit 1
timeout -k 10 200 python bench.py --steps 20 --warmup 5 --height 2048 > gpurun_out/r4/bench_stripe2.json 2> gpurun_out/r4/bench_stripe2.err || exit 1
timeout -k 10 200 python bench.py --steps 20 --warmup 5 > gpurun_out/r4/bench_n1b.json 2> gpurun_out/r4/bench_n1b.err || exit 1
