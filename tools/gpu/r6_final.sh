#!/bin/bash
# Round 6 final checkpoint: every GPU test, smoke(), the headline bench (20 steps), config 4
# (auto entropy = host on the whole box), config 4 at one rank's share (auto = GPU entropy)
set -o pipefail
export TMPDIR=/tmp
out=${1:-gpurun_out/r6y}
mkdir -p $out
CORES=$(python3 -c "import os; print(','.join(map(str, sorted(os.sched_getaffinity(0))[:2])))")
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $out/tests.txt 2>&1 || exit $?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.txt 2>&1 || exit $?
timeout -k 10 300 python bench.py --steps 20 --warmup 2 > $out/bench.json 2> $out/bench.err || exit $?
timeout -k 10 400 python bench/run.py --config 4 --out $out/c4.jsonl > $out/c4.log 2>&1 || exit $?
MIVC_ENTROPY_THREADS=2 timeout -k 10 400 taskset -c $CORES python bench/run.py --config 4 --out $out/c4_rank.jsonl > $out/c4_rank.log 2>&1 || exit $?
