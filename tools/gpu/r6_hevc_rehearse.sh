#!/bin/bash
# Round 6: config 4 batch-width sweep (--slots4 64 / 128 / 256), then configs 4 and 5 at one
# rank's share of an 8-GPU node: the process pinned to 2 of the box's cores (16 / 8) with 2 host
# CABAC threads, next to the one-rank defaults.
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r6f
mkdir -p $out
CORES=$(python3 -c "import os; print(','.join(map(str, sorted(os.sched_getaffinity(0))[:2])))")
echo "cores for the rank share: $CORES of $(python3 -c 'import os; print(len(os.sched_getaffinity(0)))')" | tee $out/info.txt
for sl in 64 128 256; do
  timeout -k 10 400 python bench/run.py --config 4 --slots4 $sl --out $out/c4_slots$sl.jsonl > $out/c4_slots$sl.log 2>&1 || exit $?
done
MIVC_ENTROPY_THREADS=2 timeout -k 10 400 taskset -c $CORES python bench/run.py --config 4 --out $out/c4_rank.jsonl > $out/c4_rank.log 2>&1 || exit $?
timeout -k 10 500 python bench/run.py --config 5 --out $out/c5_solo.jsonl > $out/c5_solo.log 2>&1 || exit $?
MIVC_ENTROPY_THREADS=2 timeout -k 10 500 taskset -c $CORES python bench/run.py --config 5 --out $out/c5_rank.jsonl > $out/c5_rank.log 2>&1 || exit $?
