#!/bin/bash
# Round 6: x264's direct / pyramid defaults on the H.264 content suite -- fast spatial direct
# (sp_tol4), the exact wavefront spatial decision (sp_wave) and wavefront spatial + b-pyramid
# (sp_wave_pyr) against the default (temporal direct, no pyramid); then the headline cost of the
# wavefront forms (same box, interleaved)
set -o pipefail
export TMPDIR=/tmp
out=${1:-gpurun_out/r6al}
mkdir -p $out
timeout -k 10 1000 python -u tools/content_rd.py run $out/h264_spatial_rd.json --configs default,sp_tol4,sp_wave,sp_wave_pyr > $out/rd.log 2>&1 || exit $?
bash tools/gpu/ab_steps.sh $out/ab 2 8 "base=" "sp_wave=MIVC_DIRECT=spatial MIVC_SPATIAL_WAVEFRONT=1" "sp_wave_pyr=MIVC_DIRECT=spatial MIVC_SPATIAL_WAVEFRONT=1 MIVC_PYRAMID=1" || exit $?
