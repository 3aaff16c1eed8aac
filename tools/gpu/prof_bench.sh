# usage: bash tools/gpu/prof_bench.sh <outdir> [bench args...]
set -o pipefail
export TMPDIR=/tmp
out=$1; shift
cd /tmp && MIVC_CABAC_GROUP=${MIVC_CABAC_GROUP:-20} timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/$out -o run -- python3 $GRAFT_REPO_ROOT/bench.py "$@" > $GRAFT_REPO_ROOT/gpurun_out/$out.log 2>&1
db=$(ls $GRAFT_REPO_ROOT/gpurun_out/$out/*.db 2>/dev/null | head -1)
[ -n "$db" ] && python3 $GRAFT_REPO_ROOT/tools/kstats.py "$db" --top 40 > $GRAFT_REPO_ROOT/gpurun_out/$out.kstats.txt 2>&1
find $GRAFT_REPO_ROOT/gpurun_out/$out -name "*.db" -delete
true
