# A/B of the unpacked RCCL device code (utils/rccl_unpack.py) on one MI355X: communicator start-up
# of tk8s-rccl with the installed library vs the unpacked copy, each in a fresh process.
set -o pipefail
out=gpurun_out/r5_rccl_unpack2
mkdir -p $out
( time timeout -k 10 300 python3 -m tritonk8ssupervisor_amd.utils.rccl_unpack ) > $out/unpack.log 2>&1 || exit $?
lib=$(python3 -c "from tritonk8ssupervisor_amd.utils.rccl_unpack import library_dir; print(library_dir() or '')")
echo "unpacked dir: $lib" >> $out/unpack.log
for i in 1 2 3; do
  timeout -k 10 120 ./tritonk8ssupervisor_amd/bin/tk8s-rccl --ngpus 1 --max-bytes 1048576 --iters 3 --warmup 1 > $out/stock_$i.json 2>> $out/err.log || exit $?
  LD_LIBRARY_PATH=$lib timeout -k 10 120 ./tritonk8ssupervisor_amd/bin/tk8s-rccl --ngpus 1 --max-bytes 1048576 --iters 3 --warmup 1 > $out/unpacked_$i.json 2>> $out/err.log || exit $?
  echo "round $i done"
done
# where the rest of the communicator start goes: RCCL's own INIT log, timestamped
NCCL_DEBUG=INFO NCCL_DEBUG_SUBSYS=INIT,ENV LD_LIBRARY_PATH=$lib timeout -k 10 120 ./tritonk8ssupervisor_amd/bin/tk8s-rccl --ngpus 1 --max-bytes 1048576 --iters 3 --warmup 1 > $out/unpacked_debug.json 2> $out/unpacked_debug.err || exit $?
