# RD sweep of one encoder knob (environment variable) over several CRFs:
#   bash tools/gpu/rd_knob.sh <outdir> <VAR> "<values>" ["<crfs>"] [extra bench.py args]
# bench.py at 1080p with 64 segments, quality measured on the first warmup step; one log per
# (value, crf) plus summary.txt lines "VAR=value crf kb/s PSNR-Y fps"
set -o pipefail
out=gpurun_out/$1; var=$2; vals=$3; crfs=${4:-"18 23 28 33"}
extra=""; if [ $# -gt 4 ]; then shift 4; extra="$*"; fi
mkdir -p $out
for v in $vals; do
  for crf in $crfs; do
    env $var=$v timeout -k 10 200 python bench.py --steps 1 --warmup 1 --slots 64 --crf $crf $extra > $out/${var}_${v}_${crf}.log 2>&1 || exit 1
    echo "$var=$v $crf $(tail -1 $out/${var}_${v}_${crf}.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); q=d["quality"]; print(q["bitrate_kbps"], q["psnr_y_db"], d["value"])')" >> $out/summary.txt
  done
done
