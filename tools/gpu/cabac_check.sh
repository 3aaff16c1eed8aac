set -o pipefail
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_h264.py -k "cabac or entropy or qps" > gpurun_out/t.log 2>&1 && \
timeout -k 10 200 python bench.py --steps 3 --warmup 1 > gpurun_out/b8.log 2>&1 && \
MIVC_CABAC_GROUP=20 timeout -k 10 200 python bench.py --steps 3 --warmup 1 > gpurun_out/b20.log 2>&1
