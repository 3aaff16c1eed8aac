#!/bin/bash
# Round 6: kernel trace of the HEVC GPU entropy stage (tools/gpu_entropy_probe.py, 64 x 8 1080p)
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
out=$R/gpurun_out/r6o
mkdir -p $out
cd /tmp
timeout -s KILL 300 rocprofv3 --kernel-trace --stats -d $out/tr -o run -- python3 $R/tools/gpu_entropy_probe.py 64 8 > $out/probe.log 2>&1 || exit $?
db=$(ls $out/tr/*/*.db $out/tr/*.db 2>/dev/null | head -1)
python3 $R/tools/kernel_calls.py "$db" hevc_entropy 40 > $out/entropy_calls.md 2>&1
python3 $R/tools/rocpd_summary.py "$db" "entropy probe 64 x 8 1080p" > $out/summary.md 2>&1
find $out -name "*.db" -delete
true
