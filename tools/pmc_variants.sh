#!/bin/bash
# One SQ --pmc pass per library variant (SLK_LIB_VARIANT), kernel driver = tools/kdriver.py.
# usage: tools/pmc_variants.sh lib1.so lib2.so ...   (results: gpurun_out/pmcv/<name>/)
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/pmcv}
for lib in "$@"; do
  name=$(basename "$lib" .so)
  mkdir -p $OUT/$name
  SLK_LIB_VARIANT=$lib timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_ANY GRBM_GUI_ACTIVE -d $OUT/$name -o sq --output-format csv -- python tools/kdriver.py ${KARGS:---steps 3} > $OUT/$name.log 2>&1
  rc=$?; echo "pass $name rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
