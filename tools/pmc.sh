#!/bin/bash
# Three separate rocprofv3 --pmc passes (the guide's slot limits; no trace domains mixed in).
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/pmc}
ARGS=${KARGS:---steps 3}
mkdir -p $OUT
run() {  # name counters...
  local name=$1; shift
  timeout -s KILL 120 rocprofv3 --pmc "$@" -d $OUT/$name -o $name --output-format csv -- python tools/kdriver.py $ARGS > $OUT/$name.log 2>&1
  local rc=$?; echo "pass $name rc=$rc"; return $rc
}
run sq SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE || exit $?
run fetch FETCH_SIZE GRBM_GUI_ACTIVE || exit $?
run write WRITE_SIZE TCC_HIT_sum TCC_MISS_sum || exit $?
