#!/usr/bin/env bash
# Where the RCCL communicator start goes with the unpacked library (utils/rccl_unpack.py): one
# tk8s-rccl run at n=1 with RCCL's INFO log timestamped to the microsecond.
set -o pipefail
out=gpurun_out/${1:-r5_rccl_init}
mkdir -p $out
lib=$(python3 -c "from tritonk8ssupervisor_amd.utils.rccl_unpack import library_dir; print(library_dir() or '')")
[ -n "$lib" ] || { echo "no unpacked RCCL (run build first)"; exit 1; }
for i in 1 2; do
  LD_LIBRARY_PATH=$lib NCCL_DEBUG=INFO NCCL_DEBUG_SUBSYS=ALL NCCL_DEBUG_TIMESTAMP_LEVELS=ALL \
    NCCL_DEBUG_TIMESTAMP_FORMAT="%H:%M:%S.%6f " TK8S_TRACE=1 \
    timeout -k 10 120 ./tritonk8ssupervisor_amd/bin/tk8s-rccl --rank 0 --nranks 1 --uid-file $out/uid$i \
      --max-bytes 1048576 --iters 3 --warmup 1 > $out/run$i.log 2>&1 || exit $?
done
echo done
