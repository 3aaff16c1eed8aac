# Kernel trace of bench/run.py, per (kernel, grid) durations for kernels matching a pattern:
#   bash tools/gpu/trace_grid.sh <outname> '<regex>' [bench/run.py args...] -> gpurun_out/<outname>.md
set -o pipefail
export TMPDIR=/tmp
out=$1; pat=$2; shift 2
R=$GRAFT_REPO_ROOT
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace -d $R/gpurun_out/$out -o run -- python3 $R/bench/run.py "$@" > $R/gpurun_out/$out.log 2>&1
rc=$?
db=$(find $R/gpurun_out/$out -name "*.db" | head -1)
[ -n "$db" ] && python3 $R/tools/kgrid.py "$db" "$pat" > $R/gpurun_out/$out.md 2>&1
find $R/gpurun_out/$out -name "*.db" -delete
exit $rc
