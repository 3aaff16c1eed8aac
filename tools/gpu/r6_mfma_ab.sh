#!/bin/bash
# Round 6: the sa8d-on-MFMA kernels -- bit-exact H.264 GPU tests, then a same-box A/B of the
# headline against the libraries without them (base: neither, interonly: t8 decision only).
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r6e
mkdir -p $out
timeout -k 10 400 python -u -m pytest tests/test_gpu_h264.py tests/test_gpu_satd.py -x -q --timeout 200 --timeout-method thread > $out/tests.txt 2>&1 || exit $?
bash tools/gpu/ab_steps.sh $out/ab 3 8 "base=MIVC_HIP_LIB=abso/base.so" "interonly=MIVC_HIP_LIB=abso/interonly.so" "mfma="
