# blur:31 / conv:31 A/B (16K RGB and the N=8 stripe), one process per variant
mkdir -p gpurun_out/r4/blur
C31="$(python3 -c "print('conv:31:' + ';'.join(str(((i*7)%13-4)/400.0) for i in range(961)))")"
for v in 0 1 2 3; do
  STRIPE_BLUR_VARIANT=$v timeout -k 10 120 python tools/kbench.py --chains "blur:31|blur:31:lsb" --shape 16384x16384x3 --iters 30 > gpurun_out/r4/blur/v${v}_16k.txt 2>&1 || exit 1
  STRIPE_BLUR_VARIANT=$v timeout -k 10 120 python tools/kbench.py --chains "blur:31|blur:31:lsb" --shape 16384x2048x3 --iters 60 > gpurun_out/r4/blur/v${v}_stripe.txt 2>&1 || exit 1
done
timeout -k 10 120 python tools/kbench.py --chains "$C31|$C31:lsb" --shape 16384x16384x3 --iters 10 > gpurun_out/r4/blur/conv31_16k.txt 2>&1 || exit 1
