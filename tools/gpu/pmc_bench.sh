# usage: [BENCH_SCRIPT=bench/run.py] BENCH_ARGS="..." bash tools/gpu/pmc_bench.sh <outdir>
# One rocprofv3 --pmc pass per counter group (each within the per-block limits: <=8 SQ,
# <=4 TCC with FETCH_SIZE = 3 and WRITE_SIZE = 2, <=2 GRBM), every pass under its own hard
# time limit; counters the device does not list are dropped; stops at the first failure.
set -o pipefail
export TMPDIR=/tmp
out=$1; shift
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/$out
cd /tmp
timeout -s KILL 60 rocprofv3 -L > $R/gpurun_out/$out/avail.txt 2>&1 || true
pass() {
  local name=$1; shift
  local keep=()
  for c in "$@"; do
    if grep -qw "$c" $R/gpurun_out/$out/avail.txt; then keep+=("$c"); fi
  done
  echo "pass $name: ${keep[*]}" >> $R/gpurun_out/$out/passes.txt
  [ ${#keep[@]} -eq 0 ] && return 0
  timeout -s KILL 240 rocprofv3 --kernel-trace --pmc "${keep[@]}" -d $R/gpurun_out/$out/$name -o run -- \
    python3 $R/${BENCH_SCRIPT:-bench.py} $BENCH_ARGS > $R/gpurun_out/$out/$name.log 2>&1
}
pass p1 SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_MFMA SQ_LDS_BANK_CONFLICT &&
pass p2 SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_LDS SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE &&
pass p3 FETCH_SIZE &&
pass p4 WRITE_SIZE
# summaries on the box (the databases are too large to copy back)
for p in p1 p2 p3 p4; do
  db=$(ls $R/gpurun_out/$out/$p/*.db 2>/dev/null | head -1)
  [ -n "$db" ] && python3 $R/tools/pmc_summary.py "$db" > $R/gpurun_out/$out/$p.summary.txt 2>&1
done
find $R/gpurun_out/$out -name "*.db" -delete
true
