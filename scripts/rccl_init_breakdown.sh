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
# RCCL start-up knobs, 3 fresh processes each: which of RCCL's optional subsystems cost start time
for variant in "BASE=1" "NCCL_IB_DISABLE=1" "RCCL_MSCCL_ENABLE=0 RCCL_MSCCLPP_ENABLE=0" "NCCL_NET_PLUGIN=none" \
               "NCCL_IB_DISABLE=1 RCCL_MSCCL_ENABLE=0 RCCL_MSCCLPP_ENABLE=0 NCCL_NET_PLUGIN=none"; do
  for i in 1 2 3; do
    env $variant LD_LIBRARY_PATH=$lib timeout -k 10 120 ./tritonk8ssupervisor_amd/bin/tk8s-rccl --ngpus 1 \
      --max-bytes 1048576 --iters 3 --warmup 1 2>/dev/null | tail -1 | \
      python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$variant', d['comm_init_ms'], d.get('sweep_ms'))" \
      >> $out/knobs.txt || exit $?
  done
done
echo knobs done
