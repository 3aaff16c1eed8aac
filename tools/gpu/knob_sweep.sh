# bench.py fps / bitrate / PSNR for encoder knob settings given as env assignments:
#   bash tools/gpu/knob_sweep.sh "MIVC_B_EARLY_SAD=0" "MIVC_B_EARLY_SAD=256" ...
set -o pipefail
for kv in "$@"; do
  tag=$(echo "$kv" | tr -c 'A-Za-z0-9_=' '_')
  env $kv timeout -k 10 200 python bench.py --allow-knobs --steps 2 --warmup 1 > gpurun_out/knob_$tag.log 2>&1 || exit 1
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().splitlines()[-1]); q=d['quality']; print(sys.argv[2], d['value'], q['bitrate_kbps'], q['psnr_y_db'])" gpurun_out/knob_$tag.log "$kv"
done
