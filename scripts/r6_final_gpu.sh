#!/bin/bash
# Round-6 GPU check of the whole tree: the GPU suite, then bench.py with an injected RCCL hang
# (the fabric check fails fast and is turned off for the rest of the steps), then the default
# bench.py run. Each step bounded; a failing step ends the script.
#   scripts/r6_final_gpu.sh OUTDIR
set -u
out=$1
mkdir -p "$out"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$out/pytest_gpu.log" 2>&1
rc=$?
echo "pytest rc=$rc" > "$out/status"
[ $rc -le 1 ] || exit $rc
TK8S_FAULTS=rccl.hang@sweep timeout -k 10 400 python bench.py --steps 20 --warmup 5 --rccl on --rccl-op-timeout 5 \
    --curve-steps 0 --plain-steps 0 --fabric-steps 0 --back-to-back 0 > "$out/bench_fault.json" 2> "$out/bench_fault.err"
rc=$?
echo "bench_fault rc=$rc" >> "$out/status"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py > "$out/bench_default.json" 2> "$out/bench_default.err"
echo "bench_default rc=$?" >> "$out/status"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$out/smoke.log" 2>&1
echo "smoke rc=$?" >> "$out/status"
