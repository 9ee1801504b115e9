#!/bin/bash
# VALU counters over the MD5 tree (256 MiB, MALL flushed before each tree): is the leaf kernel
# VALU-issue-bound? One counter pass, bounded; then the same with the fill/copy for contrast.
#   scripts/r6_md5_pmc.sh OUTDIR
set -u
R=${GRAFT_REPO_ROOT:-$PWD}
out=$(realpath -m "$1"); mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp
[ -e "$out/pmc_md5/k_counter_collection.csv" ] || timeout -s KILL 60 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE \
    --kernel-trace --stats -d "$out/pmc_md5" -o k --output-format csv -- "$R/build/kernel_rates" md5 268435456 5 \
    > "$out/pmc_md5.json" 2> "$out/pmc_md5.err" || exit $?
echo done > "$out/status"
timeout -s KILL 60 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES GRBM_GUI_ACTIVE \
    --kernel-trace --stats -d "$out/pmc_md5_wait" -o k --output-format csv -- "$R/build/kernel_rates" md5 268435456 5 \
    > "$out/pmc_md5_wait.json" 2> "$out/pmc_md5_wait.err" || exit $?
echo done2 > "$out/status"
