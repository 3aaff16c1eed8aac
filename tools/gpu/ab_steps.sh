#!/bin/bash
# Same-box A/B of bench.py settings: every setting runs `bench.py --steps S --warmup W` once per
# round, settings interleaved (A B C A B C ...), so box-to-box spread cancels.
#   [AB_ARGS="--width 3840 --height 2160 ..."] tools/gpu/ab_steps.sh OUTDIR ROUNDS STEPS "label=ENV=V ENV2=V2" "label2=" ...
set -o pipefail
export TMPDIR=/tmp
out=$1; rounds=$2; steps=$3; shift 3
mkdir -p "$out"
for r in $(seq 1 "$rounds"); do
  for spec in "$@"; do
    label=${spec%%=*}; envs=${spec#*=}
    env $envs timeout -k 10 240 python bench.py --allow-knobs --steps "$steps" --warmup 2 --no-quality $AB_ARGS > "$out/$label.r$r.log" 2>&1
    rc=$?
    echo "$label round $r rc=$rc $(grep -h '"metric"' "$out/$label.r$r.log" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); q=d["quality"]; print(d["value"], d["ms_per_step"], q.get("merged_sha256_16"), "host_blocked_s=%s" % d.get("timings_rank0_s", {}).get("host_blocked_s"), " ".join(f"{k}={v}" for k, v in d["stage_device_ms_per_step_rank0"].items() if k != "measured_on"))' 2>/dev/null)" | tee -a "$out/ab.txt"
    case $rc in 0) ;; *) exit $rc ;; esac
  done
done
