# bench.py under a list of env settings: bash tools/gpu/bench_ab.sh "A=1 B=2" "A=3" ...
set -o pipefail
export TMPDIR=/tmp
i=0
for e in "$@"; do
  env $e timeout -k 10 300 python bench.py --allow-knobs --steps 3 --warmup 1 > gpurun_out/ab$i.log 2>&1 || exit 1
  i=$((i+1))
done
