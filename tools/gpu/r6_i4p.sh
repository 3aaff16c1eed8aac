#!/bin/bash
# Round 6: Intra4x4 trials in P / B pictures (x264's default analysis): content-suite RD and a
# same-box headline A/B.
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r6h
mkdir -p $out
timeout -k 10 900 python tools/content_rd.py run $out/i4p_rd.json --configs default,i4p > $out/rd.log 2>&1 || exit $?
bash tools/gpu/ab_steps.sh $out/ab 2 8 "base=" "i4p=MIVC_I4X4_IN_P=1"
