#!/usr/bin/env bash
# A/B of the headline bench on one GPU box: the tree under gpurun_ab/old (an earlier commit, with
# the same built native tools) against the current tree, alternated so host noise hits both alike.
set -uo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/${1:-ab}"
STEPS="${2:-10}"
mkdir -p "$OUT"
export TMPDIR=/tmp
for round in ${ROUNDS:-1 2}; do
  for side in old new; do
    dir="$ROOT"; [ "$side" = old ] && dir="$ROOT/gpurun_ab/old"
    echo "[ab] round $round $side"
    (cd "$dir" && timeout -k 10 400 python3 bench.py --gpus 1 --steps "$STEPS" --warmup 3 \
        > "$OUT/${side}_${round}.json" 2> "$OUT/${side}_${round}.err") || exit $?
  done
done
echo "[ab] done"
