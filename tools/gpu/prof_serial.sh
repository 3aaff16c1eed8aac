# Isolated per-kernel cost: kernels serialised (AMD_SERIALIZE_KERNEL=3) under
# rocprofv3 --kernel-trace, summarised on the box.  usage: bash tools/gpu/prof_serial.sh <out> [bench args]
set -o pipefail
export TMPDIR=/tmp
out=$1; shift
R=$GRAFT_REPO_ROOT
export AMD_SERIALIZE_KERNEL=3
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/$out -o run -- python3 $R/bench.py "$@" > $R/gpurun_out/$out.log 2>&1
db=$(ls $R/gpurun_out/$out/*.db 2>/dev/null | head -1)
[ -n "$db" ] && python3 $R/tools/kstats.py "$db" --top 40 > $R/gpurun_out/$out.kstats.txt 2>&1
find $R/gpurun_out/$out -name "*.db" -delete
true
