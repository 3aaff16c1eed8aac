#!/bin/bash
# Round 6: HEVC GPU tests (b-adapt), HEVC b-adapt RD, Intra4x4 trials in P / B pictures (x264's
# default analysis): content-suite RD and a same-box headline A/B.
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r6h
mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_gpu_hevc.py -x -q --timeout 200 --timeout-method thread -k "badapt or multiref or inter8" > $out/tests.txt 2>&1 || exit $?
timeout -k 10 700 python tools/content_rd.py run $out/hevc_badapt_rd.json --codec hevc --configs default,ba_b2,ba_b3,ba_b3bias100,ba_b4 > $out/hrd.log 2>&1 || exit $?
timeout -k 10 700 python tools/content_rd.py run $out/i4p_rd.json --configs default,i4p > $out/rd.log 2>&1 || exit $?
bash tools/gpu/ab_steps.sh $out/ab 2 8 "base=" "i4p=MIVC_I4X4_IN_P=1"
