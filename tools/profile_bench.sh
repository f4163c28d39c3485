#!/bin/bash
# rocprofv3 passes for the round's profile evidence (run on the GPU box from the repo root):
#   1. FETCH_SIZE, WRITE_SIZE (separate passes: TCC slots) and SQ counters on the forward alone at
#      the bench's typical launch size (tools/kernel_variants.py, 512 rows, default dispatch)
#   2. kernel trace + stats of a short bench run (per-kernel average duration)
# Usage: tools/profile_bench.sh <tag> [bench args...]
set -o pipefail
TAG=${1:-r01}; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/prof_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
KV="$R/tools/kernel_variants.py --configs 2 --batches ${KV_BATCHES:-256,512} --reps 30 --variants default"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o fetch -- python3 $KV \
    > $OUT/fetch.log 2>&1 || { echo "fetch pass failed"; exit 1; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o write -- python3 $KV \
    > $OUT/write.log 2>&1 || { echo "write pass failed"; exit 1; }
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
    SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --output-format csv -d $OUT/sq -o sq -- \
    python3 $KV > $OUT/sq.log 2>&1 || { echo "sq pass failed"; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kv -o kv -- python3 $KV \
    > $OUT/kv_trace.log 2>&1 || { echo "kv trace pass failed"; exit 1; }
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o bench -- \
    python3 $R/bench.py --no-cpu-baseline "$@" > $OUT/bench_trace.log 2>&1 || { echo "trace pass failed"; exit 1; }
echo PROFILE OK
