# RD points: bench.py at several CRFs for four encoder configurations (quality measured
# on the first warmup step): High CABAC 8x8dct + 3 B, Main CABAC + 3 B, Main CABAC P-only,
# Baseline CAVLC (round 1)
set -o pipefail
export TMPDIR=/tmp
for crf in 18 23 28 33; do
  for cfg in "--bframes 3" "--bframes 3 --no-8x8dct" "--bframes 0 --no-8x8dct" "--bframes 0 --cavlc"; do
    tag=$(echo "$cfg" | tr -d ' -')
    timeout -k 10 200 python bench.py --steps 1 --warmup 1 --crf $crf $cfg > gpurun_out/rd_${crf}_${tag}.log 2>&1 || exit 1
  done
done
