# gloo-gpu rehearsals of the multi-process device path on the one-GPU box:
# N processes share GPU 0, gloo moves device buffers through pinned memory.
mkdir -p gpurun_out/r4/shared
O=gpurun_out/r4/shared
TR="python -m torch.distributed.run --nnodes=1 --master-addr 127.0.0.1"
timeout -k 10 300 $TR --nproc-per-node 4 --master-port 29541 bench.py --gpus 4 --backend gloo-gpu --steps 20 --warmup 5 > $O/bench_16k_n4.json 2> $O/bench_16k_n4.err || exit 1
timeout -k 10 400 $TR --nproc-per-node 8 --master-port 29543 bench.py --gpus 8 --backend gloo-gpu --steps 20 --warmup 5 --e2e-steps 0 --ref-steps 0 > $O/bench_16k_n8.json 2> $O/bench_16k_n8.err || exit 1
# last: a peer exits (injected, STRIPE_FAULT) in the dist scope; the headline line must still print
STRIPE_FAULT=dist@1:exit timeout -k 10 300 $TR --nproc-per-node 4 --master-port 29542 bench.py --gpus 4 --backend gloo-gpu --steps 20 --warmup 5 --comm-timeout-s 30 > $O/bench_16k_n4_fault.json 2> $O/bench_16k_n4_fault.err
echo "fault run exit $?" >> $O/bench_16k_n4_fault.err
