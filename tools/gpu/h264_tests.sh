# H.264 GPU tests (optionally a -k filter), then an optional short bench
set -o pipefail
export TMPDIR=/tmp
k=${1:-}
if [ -n "$k" ]; then
  timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_h264.py -k "$k" > gpurun_out/t.log 2>&1 || exit 1
else
  timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_h264.py > gpurun_out/t.log 2>&1 || exit 1
fi
if [ -n "${BENCH:-}" ]; then timeout -k 10 300 python bench.py --steps 3 --warmup 1 > gpurun_out/b.log 2>&1 || exit 1; fi
