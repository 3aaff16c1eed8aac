#!/bin/bash
# Round 6 checkpoint: every GPU test, smoke(), the headline bench (20 steps), config 4 and a
# headline kernel trace with its steady-state busy share.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
out=$R/gpurun_out/r6i
mkdir -p $out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $out/tests.txt 2>&1 || exit $?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.txt 2>&1 || exit $?
timeout -k 10 300 python bench.py --steps 20 --warmup 2 > $out/bench.json 2> $out/bench.err || exit $?
timeout -k 10 400 python bench/run.py --config 4 --out $out/c4.jsonl > $out/c4.log 2>&1 || exit $?
cd /tmp
timeout -s KILL 300 rocprofv3 --kernel-trace --stats -d $out/trace_h264 -o run -- python3 $R/bench.py --steps 5 --warmup 2 > $out/trace_h264.log 2>&1 || exit $?
db=$(ls $out/trace_h264/*/*.db $out/trace_h264/*.db 2>/dev/null | head -1); [ -n "$db" ] && python3 $R/tools/rocpd_summary.py "$db" "headline, bench.py --steps 5 --warmup 2" > $out/trace_h264.md 2>&1
find $out -name "*.db" -delete
true
