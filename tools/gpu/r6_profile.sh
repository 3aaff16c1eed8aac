#!/bin/bash
# Round 6 profiles: kernel traces (stream timeline) of the headline and of config 4, then PMC
# passes of the headline (MFMA / VALU / LDS counters of encode_inter_mb's sa8d) and config 4.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
out=$R/gpurun_out/r6g
mkdir -p $out
cd /tmp
timeout -s KILL 300 rocprofv3 --kernel-trace --stats -d $out/trace_h264 -o run -- python3 $R/bench.py --steps 5 --warmup 2 > $out/trace_h264.log 2>&1 || exit $?
db=$(ls $out/trace_h264/*/*.db $out/trace_h264/*.db 2>/dev/null | head -1); [ -n "$db" ] && python3 $R/tools/rocpd_summary.py "$db" "headline, bench.py --steps 5 --warmup 2" > $out/trace_h264.md 2>&1
timeout -s KILL 400 rocprofv3 --kernel-trace --stats -d $out/trace_c4 -o run -- python3 $R/bench/run.py --config 4 --steps 3 > $out/trace_c4.log 2>&1 || exit $?
db=$(ls $out/trace_c4/*/*.db $out/trace_c4/*.db 2>/dev/null | head -1); [ -n "$db" ] && python3 $R/tools/rocpd_summary.py "$db" "config 4, bench/run.py --config 4 --steps 3" > $out/trace_c4.md 2>&1
find $out -name "*.db" -delete
cd $R
BENCH_ARGS="--steps 2 --warmup 1" bash tools/gpu/pmc_bench.sh r6g/pmc_h264 || exit $?
BENCH_SCRIPT=bench/run.py BENCH_ARGS="--config 4 --steps 1 --slots4 64" bash tools/gpu/pmc_bench.sh r6g/pmc_c4
