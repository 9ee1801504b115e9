#!/bin/bash
# A/B of one environment switch on the worker curve, alternated on one box so its load drifts
# land on both arms:  scripts/r6_env_ab.sh OUTDIR "VAR=A" "VAR=B" ROUNDS WORKERS
set -u
out=$1; a=$2; b=$3; rounds=${4:-3}; workers=${5:-1,8}
mkdir -p "$out"
for i in $(seq 1 "$rounds"); do
  for arm in "$a" "$b"; do
    tag=$(echo "$arm" | tr '=' '_')
    env "$arm" timeout -k 10 300 python bench.py --steps 1 --warmup 1 --curve-steps 5 --curve-workers "$workers" \
        --plain-steps 0 --fabric-steps 0 --back-to-back 0 > "$out/${tag}_$i.json" 2> "$out/${tag}_$i.err" || exit $?
  done
done
