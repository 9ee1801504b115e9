#!/usr/bin/env bash
# Where tk8s-rccl's communicator start goes on one MI355X: HIP + HSA API trace (rocprofv3
# --hip-trace --hsa-trace --stats; no PMC counters in this run) of the fabric Job's per-node
# command on the unpacked RCCL (utils/rccl_unpack.py). Writes under gpurun_out/r5_rccl_rt/.
set -o pipefail
out=gpurun_out/r5_rccl_rt
mkdir -p $out /tmp/tk8s_rccl_rt
timeout -k 10 600 python3 -c "from tritonk8ssupervisor_amd.utils.build_native import build; build()" > $out/build.log 2>&1
lib=$(python3 -c "from tritonk8ssupervisor_amd.utils.rccl_unpack import library_dir; print(library_dir() or '')")
echo "unpacked library dir: $lib" | tee $out/summary.txt
[[ -n "$lib" ]] || exit 3
export LD_LIBRARY_PATH=$lib${LD_LIBRARY_PATH:+:$LD_LIBRARY_PATH}
# once without the profiler for the plain figure, then traced (--teardown: let the profiler flush)
timeout -k 10 120 ./tritonk8ssupervisor_amd/bin/tk8s-rccl --group-index 0 --devices 0 --nranks 1 \
  --uid-file /tmp/tk8s_rccl_rt/uid0 --max-bytes 4194304 --iters 3 --warmup 1 > $out/plain.json 2> $out/plain.err
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --hip-trace --hsa-trace --stats --output-format csv -d $out/trace -o run -- \
  ./tritonk8ssupervisor_amd/bin/tk8s-rccl --group-index 0 --devices 0 --nranks 1 --teardown \
  --uid-file /tmp/tk8s_rccl_rt/uid1 --max-bytes 4194304 --iters 3 --warmup 1 > $out/traced.json 2> $out/traced.err
echo done >> $out/summary.txt
