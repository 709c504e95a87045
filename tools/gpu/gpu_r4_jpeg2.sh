#!/bin/bash
# Progressive JPEG on one MI355X: the JPEG tests (host + GPU pixel stages) and
# jpegbench at 4K / 8K (sequential and libjpeg-progressive inputs).
set -o pipefail
O=gpurun_out/r4/jpeg2
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_jpeg.py -x -q --timeout 120 --timeout-method thread > $O/tests_jpeg.txt 2>&1 || exit 1
timeout -k 10 300 python tools/jpegbench.py --size 4096 > $O/jpeg_4k.json 2>&1 || exit 1
timeout -k 10 300 python tools/jpegbench.py --size 8192 > $O/jpeg_8k.json 2>&1 || exit 1
echo done
