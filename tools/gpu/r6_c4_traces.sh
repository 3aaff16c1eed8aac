#!/bin/bash
# Round 6: final config-4 kernel traces (whole box: host entropy; rank share: GPU entropy on the
# copy stream), with the steady-state busy share (tools/rocpd_summary.py)
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
out=$R/gpurun_out/r6ab
mkdir -p $out
cd /tmp
timeout -s KILL 400 rocprofv3 --kernel-trace --stats -d $out/c4 -o run -- python3 $R/bench/run.py --config 4 --out $out/c4.jsonl > $out/c4.log 2>&1 || exit $?
db=$(ls $out/c4/*/*.db $out/c4/*.db 2>/dev/null | head -1); python3 $R/tools/rocpd_summary.py "$db" "config 4, bench/run.py --config 4 (256 x 30 1080p, host entropy)" > $out/c4_trace.md 2>&1
find $out -name "*.db" -delete
MIVC_HEVC_ENTROPY=gpu timeout -s KILL 400 rocprofv3 --kernel-trace --stats -d $out/c4g -o run -- python3 $R/bench/run.py --config 4 --out $out/c4g.jsonl > $out/c4g.log 2>&1 || exit $?
db=$(ls $out/c4g/*/*.db $out/c4g/*.db 2>/dev/null | head -1); python3 $R/tools/rocpd_summary.py "$db" "config 4 with GPU entropy (MIVC_HEVC_ENTROPY=gpu)" > $out/c4g_trace.md 2>&1
find $out -name "*.db" -delete
true
