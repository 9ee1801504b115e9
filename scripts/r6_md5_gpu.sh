#!/bin/bash
# The fan-in-4 MD5 tree on the MI355X: the kernel tests (hashlib oracle, both probes' pinned
# digest), each piece event-timed alone (build/md5_roofline), then the tree under rocprofv3.
#   scripts/r6_md5_gpu.sh OUTDIR
set -u
R=${GRAFT_REPO_ROOT:-$PWD}
out=$(realpath -m "$1"); mkdir -p "$out"
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py \
    > "$out/pytest_kernels_gpu.log" 2>&1 || exit $?
timeout -k 10 120 "$R/build/md5_roofline" 256 30 > "$out/md5_roofline_256m.jsonl" 2> "$out/md5_roofline.err" || exit $?
timeout -k 10 120 "$R/build/md5_roofline" 1024 20 > "$out/md5_roofline_1g.jsonl" 2>> "$out/md5_roofline.err" || exit $?
cd /tmp && export TMPDIR=/tmp
for b in $((256 << 20)) $((1 << 30)); do
  timeout -k 10 90 rocprofv3 --kernel-trace --stats -d "$out/trace_md5_$b" -o k --output-format csv -- \
      "$R/build/kernel_rates" md5 "$b" 20 > "$out/rates_md5_$b.json" 2> "$out/rates_md5_$b.err" || exit $?
done
echo done > "$out/status"
