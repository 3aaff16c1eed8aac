#!/bin/bash
# Round 6: x265 --tu-inter-depth 1 and --signhide on the content suite (HEVC), plus the config-4
# throughput of tu-inter-depth 1
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r6af
mkdir -p $out
timeout -k 10 900 python tools/content_rd.py run $out/hevc_tud_rd.json --codec hevc --configs default,tud1,sdh > $out/rd.log 2>&1 || exit $?
bash tools/gpu/ab_config4.sh $out/ab4 2 "base=" "tud1=MIVC_HEVC_TU_INTER_DEPTH=1" || exit $?
