#!/bin/bash
# Per-rank resource rehearsal on a one-GPU box (round-5 review item): what one rank of an
# 8-GPU node would get -- a pinned-memory budget of host RAM / 32 (runtime/device.py gives each of
# 8 ranks a quarter of host RAM / 8) and cores / 8 entropy threads -- against the one-rank
# defaults, plus tighter thread counts, interleaved on one box:
#   bash tools/gpu/rehearse_rank.sh OUTDIR STEPS
set -o pipefail
out=$1; steps=${2:-20}
mkdir -p "$out"
budget=$(python3 -c 'from govideocompressor_amd.runtime.device import host_mem_total as h; print(h() // 32 // (1 << 20))')
cores=$(nproc)
thr=$(( cores / 8 )); [ $thr -gt 16 ] && thr=16; [ $thr -lt 1 ] && thr=1
echo "host_mem_MB=$(python3 -c 'from govideocompressor_amd.runtime.device import host_mem_total as h; print(h() >> 20)') cores=$cores rank_budget_MB=$budget rank_threads=$thr" | tee "$out/env.txt"
bash tools/gpu/ab_steps.sh "$out" 1 "$steps" "solo=" "rank8=MIVC_PINNED_BUDGET_MB=$budget MIVC_ENTROPY_THREADS=$thr" \
  "thr8=MIVC_PINNED_BUDGET_MB=$budget MIVC_ENTROPY_THREADS=8" "thr4=MIVC_PINNED_BUDGET_MB=$budget MIVC_ENTROPY_THREADS=4"
