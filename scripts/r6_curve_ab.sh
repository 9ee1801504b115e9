#!/bin/bash
# Worker-curve A/B on one box: the current tree and the round-4 tree (build/r4tree,
# a git-ignored copy) alternated, so box load drifts land on both.
#   scripts/r6_curve_ab.sh OUTDIR ROUNDS
set -u
out=$1; rounds=${2:-2}
mkdir -p "$out"
R=$PWD
for i in $(seq 1 "$rounds"); do
  timeout -k 10 300 python bench.py --steps 1 --warmup 1 --curve-steps 5 --plain-steps 0 --fabric-steps 0 \
      --back-to-back 0 --keep-events "$out/ev_new$i" > "$out/new$i.json" 2> "$out/new$i.err" || exit $?
  (cd build/r4tree && timeout -k 10 300 python bench.py --steps 1 --warmup 1 --curve-steps 5 --back-to-back 0 \
      > "$R/$out/r4_$i.json" 2> "$R/$out/r4_$i.err") || exit $?
done
