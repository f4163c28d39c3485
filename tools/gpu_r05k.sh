#!/bin/bash
# r05k: games/s for configs 3-5.
#   cfg3: the bench's command on reversi 10x128 (games complete in the window; GPU busy re-measured)
#   len4 / len5: hexLG13 / amazons with few game slots (16 threads x 1 pool x 1 game) run ~17 min so
#     every slot's first game completes: E[evals per game] for the renewal estimate
#     games/s = (the config's bench rate) / E[evals per game]
set -o pipefail
TAG=${1:-r05k}; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
T=$R/gpurun_out/$TAG
mkdir -p $T
cd $R
summ() {
  python - "$1" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
c = d["per_game_cost"]["first_game_cohort"]
print(sys.argv[1].split("/")[-1], "%.4g leaf-evals/s %.3g games/s busy %.3f" % (d["value"], d["games_per_sec"], d["gpu_busy_frac"]),
      "cohort completed %d in progress %d" % (c["completed"], c["in_progress"]), c.get("games_per_sec_renewal"))
PY
}
for n in "$@"; do
  case $n in
    cfg3) timeout -k 10 620 python -u bench.py --config 3 --steps 10 --warmup 2 > $T/bench_cfg3.log 2>&1 || { echo "cfg3 failed"; tail -5 $T/bench_cfg3.log; exit 1; }
          summ $T/bench_cfg3.log ;;
    len4) timeout -k 10 1150 python -u bench.py --config 4 --pools 1 --batch 1 --age-games 1000 --age-seconds 1000 --steps 2 --warmup 0 --step-rows 16384 --no-cpu-baseline > $T/len_cfg4.log 2>&1 || { echo "len4 failed"; tail -5 $T/len_cfg4.log; exit 1; }
          summ $T/len_cfg4.log ;;
    len5) timeout -k 10 1150 python -u bench.py --config 5 --pools 1 --batch 1 --age-games 1000 --age-seconds 1000 --steps 2 --warmup 0 --step-rows 16384 --no-cpu-baseline > $T/len_cfg5.log 2>&1 || { echo "len5 failed"; tail -5 $T/len_cfg5.log; exit 1; }
          summ $T/len_cfg5.log ;;
  esac
done
