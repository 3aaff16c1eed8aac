# kernel + memory-copy trace of a short bench (no counters)
set -o pipefail
export TMPDIR=/tmp
out=$1; shift
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d $GRAFT_REPO_ROOT/gpurun_out/$out -o run -- python3 $GRAFT_REPO_ROOT/bench.py "$@" > $GRAFT_REPO_ROOT/gpurun_out/$out.log 2>&1
