#!/bin/bash
# PMC passes of the split trunk at the bench's launch size (1024 rows): FETCH_SIZE | WRITE_SIZE |
# SQ counters + GRBM_GUI_ACTIVE (active cycles summed over the 8 XCDs: the MFMA-busy denominator),
# each its own rocprofv3 run (gpurun refuses combining --pmc with the trace domains)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-pmc_r04}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
KV="$R/tools/kernel_variants.py --configs 2 --batches 1024 --reps 30 --variants default --precision bf16x3"
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o fetch -- python3 $KV > $OUT/fetch.log 2>&1 || { echo "fetch pass failed"; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o write -- python3 $KV > $OUT/write.log 2>&1 || { echo "write pass failed"; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
    SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE --output-format csv -d $OUT/sq -o sq -- \
    python3 $KV > $OUT/sq.log 2>&1 || { echo "sq pass failed"; exit 1; }
python3 $R/tools/pmc_summary.py $(find $OUT -name "*counter_collection.csv") > $OUT/summary.txt
find $OUT -name "*counter_collection.csv" -size +2M -delete
cat $OUT/summary.txt
echo PMC OK
