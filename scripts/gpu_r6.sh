#!/bin/bash
# Round-6 GPU check: a pytest selection (-m gpu), then -- only if pytest ended normally (passed,
# failed or selected nothing; never after a time limit, abort or crash) -- bench.py with the
# given arguments. Every step has its own time limit.
#   scripts/gpu_r6.sh OUTDIR "BENCH ARGS" PYTEST_TARGETS...
out=$1; bargs=$2; shift 2
mkdir -p "$out"
if [ $# -gt 0 ]; then
  timeout -k 10 420 python -u -m pytest "$@" -v --timeout 180 --timeout-method thread -m gpu > "$out/pytest.log" 2>&1
  rc=$?
  echo "pytest rc=$rc" > "$out/status"
  case $rc in 0|1|5) ;; *) exit $rc ;; esac
fi
[ "$bargs" = "none" ] && exit 0
timeout -k 10 540 python -u bench.py $bargs > "$out/bench.json" 2> "$out/bench.err"
rc=$?
echo "bench rc=$rc" >> "$out/status"
exit $rc
