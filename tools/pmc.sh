#!/bin/bash
# PMC passes over the bench of config CFG (default C3) (graph replay, no eager profiling) and the FETCH/WRITE
# calibration kernel.  Counter passes run with counter collection only (no tracing domains),
# each under its own time limit; any failure ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/pmc_${CFG:-C3}
mkdir -p $OUT
BENCH="python3 bench.py --config ${CFG:-C3} --steps ${STEPS:-5} --warmup 1 --no-cpu-baseline --prof-steps 0 --settle-ms 0"
pass() {  # pass <name> <counters...>
  local name=$1; shift
  timeout -k 10 300 rocprofv3 --pmc "$@" -d $OUT/$name -o $name --output-format csv -- $BENCH \
    > $OUT/$name.log 2>&1 || { echo "pmc pass $name failed rc=$?"; tail -5 $OUT/$name.log; exit 3; }
  echo "pass $name ok"
}
cal() {  # cal <name> <counter>
  timeout -k 10 120 rocprofv3 --pmc "$2" -d $OUT/$1 -o $1 --output-format csv -- tools/calib/calib_fetch \
    > $OUT/$1.log 2>&1 || { echo "calib $1 failed"; tail -5 $OUT/$1.log; exit 3; }
  echo "calib $1 ok"
}
cal cal_fetch FETCH_SIZE
cal cal_write WRITE_SIZE
pass fetch FETCH_SIZE
pass write WRITE_SIZE
for p in ${PASSES:-sq1 sq2 tcc}; do
  case $p in
    sq1) pass sq1 SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_INSTS_VALU ;;
    sq2) pass sq2 SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU_FLOPS_FP64 SQ_INSTS_SMEM ;;
    tcc) pass tcc TCC_HIT_sum TCC_MISS_sum ;;
  esac
done
