# RD sweep of whole encoder configurations given as "name|VAR=v VAR=v ..." (bench.py knobs in the
# environment) over several CRFs:
#   bash tools/gpu/rd_cfgs.sh <outdir> "<crfs>" "r2|MIVC_REFS=1 MIVC_B_GATE=0" "r3|" ...
# summary.txt lines "name crf kb/s PSNR-Y fps" (tools/bd_knob.py reads them)
set -o pipefail
out=gpurun_out/$1; crfs=$2; shift 2
mkdir -p $out
for spec in "$@"; do
  name=${spec%%|*}; envs=${spec#*|}
  for crf in $crfs; do
    env $envs timeout -k 10 200 python bench.py --allow-knobs --steps 1 --warmup 1 --slots 64 --crf $crf > $out/${name}_${crf}.log 2>&1 || exit 1
    echo "$name $crf $(tail -1 $out/${name}_${crf}.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); q=d["quality"]; print(q["bitrate_kbps"], q["psnr_y_db"], d["value"])')" >> $out/summary.txt
  done
done
