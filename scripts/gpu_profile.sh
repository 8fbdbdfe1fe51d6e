#!/bin/bash
# rocprofv3 passes over a short bench run: kernel trace/stats, then PMC counters in separate
# passes (never combined with tracing domains).  Stops at the first crash/timeout.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp PYTHONDONTWRITEBYTECODE=1
OUT=gpurun_out/prof
mkdir -p $OUT
ARGS="bench.py --steps ${STEPS:-3} --warmup 1 --no-cpu --latency-iters 0 ${EXTRA:-}"
run() {  # name, rocprof args...
  local name=$1; shift
  timeout -k 10 300 rocprofv3 "$@" -d $OUT/$name -o $name --output-format csv -- python3 $ARGS > $OUT/$name.log 2>&1
  local rc=$?
  echo "pass $name rc=$rc"; tail -2 $OUT/$name.log
  case $rc in 124|134|137|139) exit $rc;; esac
  return 0
}
run trace --kernel-trace --stats
[ -n "$TRACE_ONLY" ] && exit 0
run pmc1 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES GRBM_GUI_ACTIVE
run pmc2 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_SALU GRBM_GUI_ACTIVE
run pmc3 --pmc FETCH_SIZE
run pmc4 --pmc WRITE_SIZE
run pmc5 --pmc TCC_HIT_sum TCC_MISS_sum SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE
python3 scripts/pmc_summary.py $OUT --json $OUT/pmc_summary.json --top 12 > $OUT/pmc_summary.txt 2>&1
exit 0
