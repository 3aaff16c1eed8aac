set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r6c
timeout -k 10 600 python tools/content_rd.py run gpurun_out/r6c/hevc_ref_rd.json --codec hevc --configs default,ref2,ref3,ref3g0,ref3g6000 > gpurun_out/r6c/rd.log 2>&1 || exit $?
bash tools/gpu/ab_config4.sh gpurun_out/r6c/ab 2 "ref1=" "ref3=MIVC_HEVC_REFS=3" "ref3g0=MIVC_HEVC_REFS=3 MIVC_HEVC_REF_GATE=0"
