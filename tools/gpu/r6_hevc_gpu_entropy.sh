#!/bin/bash
# Round 6: HEVC CABAC on the GPU (kernels/hevc_entropy.hip).  Config 4 (1080p HEVC) with host
# and GPU entropy on the same box, configs 4 and 5 at one rank's share of an 8-GPU node (2 host
# cores, 2 entropy threads: auto placement picks the GPU), as profiles/r6_hevc_rank_rehearsal.md.
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r6u
mkdir -p $out
(while sleep 50; do date >> $out/heartbeat.txt; done) &
HB=$!
trap 'kill $HB' EXIT
CORES=$(python3 -c "import os; print(','.join(map(str, sorted(os.sched_getaffinity(0))[:2])))")
echo "cores for the rank share: $CORES" | tee $out/info.txt
MIVC_HEVC_ENTROPY=host timeout -k 10 400 python bench/run.py --config 4 --out $out/c4_host.jsonl > $out/c4_host.log 2>&1 || exit $?
MIVC_HEVC_ENTROPY=gpu timeout -k 10 400 python bench/run.py --config 4 --out $out/c4_gpu.jsonl > $out/c4_gpu.log 2>&1 || exit $?
MIVC_ENTROPY_THREADS=2 timeout -k 10 400 taskset -c $CORES python bench/run.py --config 4 --out $out/c4_rank_auto.jsonl > $out/c4_rank_auto.log 2>&1 || exit $?
MIVC_ENTROPY_THREADS=2 timeout -k 10 600 taskset -c $CORES python bench/run.py --config 5 --out $out/c5_rank_auto.jsonl > $out/c5_rank_auto.log 2>&1 || exit $?
