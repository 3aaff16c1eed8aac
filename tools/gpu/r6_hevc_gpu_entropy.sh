#!/bin/bash
# Round 6: HEVC CABAC on the GPU (kernels/hevc_entropy.hip).  The HEVC GPU tests, then config 4
# (1080p HEVC) with GPU vs host entropy on the same box, and config 4 at one rank's share of an
# 8-GPU node (2 host cores, 2 entropy threads), as profiles/r6_hevc_rank_rehearsal.md.
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r6l
mkdir -p $out
CORES=$(python3 -c "import os; print(','.join(map(str, sorted(os.sched_getaffinity(0))[:2])))")
echo "cores for the rank share: $CORES" | tee $out/info.txt
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_hevc.py -k "entropy or async or multiref" > $out/tests.txt 2>&1 || exit $?
timeout -k 10 400 python bench/run.py --config 4 --out $out/c4_gpu.jsonl > $out/c4_gpu.log 2>&1 || exit $?
: MIVC_HEVC_ENTROPY=host timeout -k 10 400 python bench/run.py --config 4 --out $out/c4_host.jsonl > $out/c4_host.log 2>&1 || exit $?
MIVC_ENTROPY_THREADS=2 timeout -k 10 400 taskset -c $CORES python bench/run.py --config 4 --out $out/c4_rank_gpu.jsonl > $out/c4_rank_gpu.log 2>&1 || exit $?
