#!/bin/bash
# Same-box A/B of config 4 (1080p HEVC CRF 26) between kernel libraries / settings:
#   tools/gpu/ab_config4.sh OUTDIR ROUNDS "label=ENV=V ..." "label2=" ...
# e.g. "base=MIVC_HIP_LIB=abso/base.so" (tools/build_variant.py base --rev HEAD) against "new=".
# Settings interleaved per round so box drift cancels; one line per run in OUTDIR/ab.txt.
set -o pipefail
export TMPDIR=/tmp
out=$1; rounds=$2; shift 2
mkdir -p "$out"
for r in $(seq 1 "$rounds"); do
  for spec in "$@"; do
    label=${spec%%=*}; envs=${spec#*=}
    env $envs timeout -k 10 400 python bench/run.py --config 4 --allow-knobs --steps 3 --warmup 1 > "$out/$label.r$r.log" 2>&1
    rc=$?
    echo "$label round $r rc=$rc $(grep -h '"config": 4' "$out/$label.r$r.log" | tail -1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d.get("kbps_per_stream"), d.get("psnr_y_warmup"), d.get("ms_per_step"))' 2>/dev/null)" | tee -a "$out/ab.txt"
    case $rc in 0) ;; *) exit $rc ;; esac
  done
done
