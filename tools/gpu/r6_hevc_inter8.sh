#!/bin/bash
# Round 6: config-4 A/B of the HEVC transform variants, the 8x8-inter-CU RD sweep on the content
# suite, and config 3 at one rank's share of an 8-GPU node.
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r6d
mkdir -p $out
bash tools/gpu/ab_config4.sh $out/ab4 2 "base=MIVC_HIP_LIB=abso/base.so" "dct_nocap=MIVC_HIP_LIB=abso/dct_nocap.so" "dct_cap3=" "i8o16=MIVC_HEVC_INTER8=1 MIVC_HEVC_INTER8_OVERHEAD=16" || exit $?
timeout -k 10 700 python tools/content_rd.py run $out/hevc_inter8_rd.json --codec hevc --configs default,i8o8,i8o16,i8o24,i8o16m1000 > $out/rd.log 2>&1 || exit $?
# config 3 at one rank's share of an 8-GPU node (32 pieces, 2 parse threads = the box's 16 / 8)
# next to the whole-node-on-one-GPU shape (256 pieces, default threads)
timeout -k 10 300 python bench/run.py --config 3 --codec3 h264,hevc --segments3 32 --threads3 2 --out $out/c3_share.jsonl > $out/c3_share.log 2>&1 || exit $?
timeout -k 10 400 python bench/run.py --config 3 --codec3 h264,hevc --out $out/c3_full.jsonl > $out/c3_full.log 2>&1 || exit $?
