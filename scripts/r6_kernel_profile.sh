#!/bin/bash
# Round-6 kernel profile: every production launcher at ONE size per rocprofv3 run
# (build/kernel_rates, native/bench/kernel_rates.hip), so each kernel_stats.csv holds exactly that
# kernel at that size (the untimed warm-up is a 1 MiB launch, a row of its own in the trace);
# then FETCH_SIZE and WRITE_SIZE, each in its own --pmc pass, over our copy and the runtime's own
# device-to-device memcpy (the control with known bytes).
#   scripts/r6_kernel_profile.sh OUTDIR
set -u
R=${GRAFT_REPO_ROOT:-$PWD}
out=$(realpath -m "$1")
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp
G=$((1 << 30)); M256=$((256 << 20))
for spec in "fill $G" "fill_nt $G" "memset $G" "verify $G" "copy $G" "memcpy $G" "copy $M256" "md5 $M256" "philox $M256"; do
  set -- $spec
  timeout -k 10 90 rocprofv3 --kernel-trace --stats -d "$out/trace_$1_$2" -o k --output-format csv -- \
      "$R/build/kernel_rates" "$1" "$2" 20 > "$out/rates_$1_$2.json" 2> "$out/rates_$1_$2.err" || exit $?
done
for kind in copy memcpy verify; do
  for ctr in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 60 rocprofv3 --pmc "$ctr" --kernel-trace --stats -d "$out/pmc_${kind}_$ctr" -o k \
        --output-format csv -- "$R/build/kernel_rates" "$kind" "$G" 3 > "$out/pmc_${kind}_$ctr.json" 2>&1 || exit $?
  done
done
echo done > "$out/status"
