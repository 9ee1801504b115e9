#!/bin/bash
# RCCL start-up A/B on one GPU: which environment switches shorten the fabric Job rank's
# unique-id and communicator start (the unpacked library, huge-page malloc, as the Job runs it).
#   scripts/r6_rccl_env_ab.sh OUTDIR
set -u
out=$(realpath -m "$1"); mkdir -p "$out"
R=$PWD
timeout -k 10 600 python -c "from tritonk8ssupervisor_amd.utils.build_native import build; build()" > "$out/build.log" 2>&1 || exit $?
LIB=$R/build/rccl-gfx950
for round in 1 2 3; do
  for v in base ib_off lo both; do
    case $v in
      base) extra=() ;;
      ib_off) extra=(NCCL_IB_DISABLE=1) ;;
      lo) extra=(NCCL_SOCKET_IFNAME=lo) ;;
      both) extra=(NCCL_IB_DISABLE=1 NCCL_SOCKET_IFNAME=lo) ;;
    esac
    sleep 1
    env "${extra[@]}" TK8S_TRACE=1 LD_LIBRARY_PATH=$LIB:${LD_LIBRARY_PATH:-} GLIBC_TUNABLES=glibc.malloc.hugetlb=1 \
      timeout -k 10 60 $R/tritonk8ssupervisor_amd/bin/tk8s-rccl --rank 0 --nranks 1 --device 0 --uid-file "$out/uid_${v}_$round" --max-bytes 1024 --iters 1 --warmup 1 \
      --dtype float32 > "$out/${v}_$round.json" 2> "$out/${v}_$round.err" || exit $?
  done
done
