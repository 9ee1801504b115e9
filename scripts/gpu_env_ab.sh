#!/usr/bin/env bash
# A/B of the headline bench on one GPU box between two environments (a shortcut's off-switch,
# say), alternated so host noise hits both alike:  gpu_env_ab.sh OUT STEPS "A_ENV" "B_ENV"
# e.g. gpu_env_ab.sh lazy_ab 10 "" "TK8S_LAZY_STDLIB=0"
set -uo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/${1:-env_ab}"
STEPS="${2:-10}"
A="${3:-}"
B="${4:-}"
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$ROOT"
for round in ${ROUNDS:-1 2}; do
  for side in a b; do
    envs="$A"; [ "$side" = b ] && envs="$B"
    echo "[ab] round $round $side ($envs)"
    env $envs timeout -k 10 400 python3 bench.py --gpus 1 --steps "$STEPS" --warmup 2 --curve-steps 0 \
        --plain-steps 0 --fabric-steps 0 > "$OUT/${side}_${round}.json" 2> "$OUT/${side}_${round}.err" || exit $?
  done
done
echo "[ab] done"
