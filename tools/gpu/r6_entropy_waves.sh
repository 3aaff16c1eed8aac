#!/bin/bash
# Round 6: GPU entropy waves per picture (MIVC_HEVC_ENTROPY_WAVES 16 / 8 / 4) on config 4 with
# GPU entropy, interleaved, plus the host writer for reference
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r6x
mkdir -p $out
for r in 1 2; do
  for wv in 16 8 4; do
    MIVC_HEVC_ENTROPY=gpu MIVC_HEVC_ENTROPY_WAVES=$wv timeout -k 10 400 python bench/run.py --config 4 --out $out/c4_w$wv.r$r.jsonl > $out/c4_w$wv.r$r.log 2>&1 || exit $?
  done
done
