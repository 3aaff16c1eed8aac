#!/bin/bash
# Round 6: HEVC GPU tests, then the 8x8-inter-CU RD sweep on the content suite and a config-4 A/B.
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r6d
mkdir -p $out
timeout -k 10 400 python -u -m pytest tests/test_gpu_hevc.py -x -q --timeout 200 --timeout-method thread > $out/tests.txt 2>&1 || exit $?
timeout -k 10 700 python tools/content_rd.py run $out/hevc_inter8_rd.json --codec hevc --configs default,i8o8,i8o16,i8o24,i8o16m1000 > $out/rd.log 2>&1 || exit $?
bash tools/gpu/ab_config4.sh $out/ab 2 "base=" "i8o16=MIVC_HEVC_INTER8=1 MIVC_HEVC_INTER8_OVERHEAD=16"
# config 3 at one rank's share of an 8-GPU node (32 pieces, 2 parse threads = the box's 16 / 8)
# next to the whole-node-on-one-GPU shape (256 pieces, default threads)
timeout -k 10 300 python bench/run.py --config 3 --codec3 h264,hevc --segments3 32 --threads3 2 --out $out/c3_share.jsonl > $out/c3_share.log 2>&1 || exit $?
timeout -k 10 400 python bench/run.py --config 3 --codec3 h264,hevc --out $out/c3_full.jsonl > $out/c3_full.log 2>&1 || exit $?
