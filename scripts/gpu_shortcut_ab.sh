#!/usr/bin/env bash
# What each start-up shortcut buys on the MI355X (docs/architecture.md's table):
# the headline with all of them on, with each one off alone, and with all off (TK8S_SHORTCUTS=0),
# 10 timed steps each, the whole set repeated so host noise hits every variant alike.
set -uo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/${1:-shortcut_ab}"
STEPS="${2:-10}"
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$ROOT"
variants=("none" "TK8S_HOST_BURNIN=0" "TK8S_CP_ZYGOTE=0" "TK8S_AGENT_ZYGOTE=0"
          "TK8S_HSA_CPU_CACHES=1" "TK8S_YAML_CACHE=off" "TK8S_NO_PYCACHE_PREFIX=1"
          "TK8S_PLAY_INLINE=0" "TK8S_INPROCESS_BOOTSTRAP=0" "TK8S_FAST_ARGS=0"
          "TK8S_SKIP_SITE=0" "TK8S_SHORTCUTS=0")
[ -n "${VARIANTS:-}" ] && read -ra variants <<< "$VARIANTS"   # a subset: VARIANTS="none TK8S_X=0 ..."
CURVE=(--curve-steps "${CURVE_STEPS:-0}")
[ -n "${CURVE_WORKERS:-}" ] && CURVE+=(--curve-workers "$CURVE_WORKERS")
for round in ${ROUNDS:-1 2}; do
  for v in "${variants[@]}"; do
    tag=$(echo "$v" | tr '=' '_')
    envs="$v"; [ "$v" = none ] && envs="TK8S_AB_BASELINE=1"
    echo "[ab] round $round $v"
    env $envs timeout -k 10 300 python3 bench.py --gpus 1 --steps "$STEPS" --warmup 2 "${CURVE[@]}" \
        --plain-steps 0 --fabric-steps 0 > "$OUT/${tag}_${round}.json" 2> "$OUT/${tag}_${round}.err" || exit $?
  done
done
echo "[ab] done"
