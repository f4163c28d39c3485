#!/bin/bash
# r05h: host-engine A/B on the box's CPU (EPYC 9575F), the bench's workload aged 240 s:
#   base: x86-64-v3 engine (no PGO: the profiles are stale), scalar spin loops
#   vec : the same library, AVX2 spin loops (GZ_SPIN_VEC=1)
#   v4  : x86-64-v4 (AVX-512) build of the engine (lib_v4), scalar spin loops
#   blk : the AVX2 spin loops in blocks of eight playouts (GZ_SPIN_VEC=2)
set -o pipefail
TAG=${1:-r05h}
R=${GRAFT_REPO_ROOT:-$(pwd)}
T=$R/gpurun_out/$TAG
mkdir -p $T
cd $R
ARGS="--steps 8 --warmup 2 --age-games 3 --age-seconds 240 --no-cpu-baseline"
run() {   # name, env...
  local n=$1; shift
  env "$@" timeout -k 10 420 python -u bench.py $ARGS > $T/bench_$n.log 2>&1 || { echo "$n failed"; tail -5 $T/bench_$n.log; return 1; }
  python - "$T/bench_$n.log" "$n" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
hb = d["host_budget"]
print("%-5s %.4g leaf-evals/s  %.1f games/s  busy %.3f  per-thread %.4g  nnfree/leaf %.0f  %s" % (
    sys.argv[2], d["value"], d["games_per_sec"], d["gpu_busy_frac"], hb["leaf_evals_per_s_per_engine_thread"],
    d["nn_free_playouts_per_leaf"], d.get("engine_build")))
PY
}
for n in "$@"; do
  case $n in
    base) run base GZ_SPIN_VEC=0 || exit 1 ;;
    vec) run vec GZ_SPIN_VEC=1 || exit 1 ;;
    v4) run v4 GZ_SPIN_VEC=0 GZ_LIB_DIR=$R/galvanise_zero_amd/lib_v4 || exit 1 ;;
    v4vec) run v4vec GZ_SPIN_VEC=1 GZ_LIB_DIR=$R/galvanise_zero_amd/lib_v4 || exit 1 ;;
    blk) run blk GZ_SPIN_VEC=2 || exit 1 ;;
  esac
done
