#!/bin/bash
# Round 6: the matrix-core kernels -- bit-exact H.264 / HEVC GPU tests, then same-box A/Bs of the
# headline (base: neither sa8d on MFMA, interonly: the t8 decision only) and of config 4 (base:
# the HEVC transforms on the LDS wave products).
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r6e
mkdir -p $out
timeout -k 10 500 python -u -m pytest tests/test_gpu_h264.py tests/test_gpu_satd.py tests/test_gpu_hevc.py -x -q --timeout 200 --timeout-method thread > $out/tests.txt 2>&1 || exit $?
bash tools/gpu/ab_steps.sh $out/ab 3 8 "base=MIVC_HIP_LIB=abso/base.so" "interonly=MIVC_HIP_LIB=abso/interonly.so" "mfma=" || exit $?
bash tools/gpu/ab_config4.sh $out/ab4 2 "base=MIVC_HIP_LIB=abso/base.so" "mfma="
