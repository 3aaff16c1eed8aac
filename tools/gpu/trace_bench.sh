# Kernel trace of bench.py with the per-stream timeline summary, on the GPU box:
#   bash tools/gpu/trace_bench.sh <outname> [bench args...]  -> gpurun_out/<outname>.md
set -o pipefail
export TMPDIR=/tmp
out=$1; shift
R=$GRAFT_REPO_ROOT
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/$out -o run -- python3 $R/bench.py "$@" > $R/gpurun_out/$out.log 2>&1
rc=$?
db=$(find $R/gpurun_out/$out -name "*.db" | head -1)
[ -n "$db" ] && python3 $R/tools/rocpd_summary.py "$db" "bench.py $* kernel trace" > $R/gpurun_out/$out.md 2>&1
find $R/gpurun_out/$out -name "*.db" -delete
exit $rc
