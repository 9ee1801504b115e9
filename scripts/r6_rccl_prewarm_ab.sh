#!/bin/bash
# The fabric rank's RCCL code prewarm (tk8s_rccl.cpp prewarm_rccl_code) on and off, alternated:
# main -> sweep done, the unique id and the communicator start, from each run's TRACE lines.
#   scripts/r6_rccl_prewarm_ab.sh OUTDIR [ROUNDS]
set -u
out=$(realpath -m "$1"); rounds=${2:-4}; mkdir -p "$out"
R=$PWD
timeout -k 10 600 python -c "from tritonk8ssupervisor_amd.utils.build_native import build; build()" > "$out/build.log" 2>&1 || exit $?
LIB=$R/build/rccl-gfx950
for round in $(seq 1 "$rounds"); do
  for v in 1 0; do
    sleep 1
    TK8S_RCCL_PREWARM=$v TK8S_TRACE=1 LD_LIBRARY_PATH=$LIB:${LD_LIBRARY_PATH:-} GLIBC_TUNABLES=glibc.malloc.hugetlb=1 \
      timeout -k 10 60 $R/tritonk8ssupervisor_amd/bin/tk8s-rccl --rank 0 --nranks 1 --device 0 \
      --uid-file "$out/uid_${v}_$round" --min-bytes 1024 --max-bytes 67108864 --factor 4 --iters 5 --warmup 2 \
      --dtype float32 > "$out/prewarm${v}_$round.json" 2> "$out/prewarm${v}_$round.err" || exit $?
  done
done
