#!/bin/bash
# tk8s-gpuinfo on the MI355X: on the host, then inside a synthetic image in ptrace mode (without
# and with the GPU jail), each run's translated syscalls logged (TK8S_PTRACE_LOG).
#   scripts/r6_ptrace_gpu_debug.sh OUTDIR
set -u
out=$(realpath -m "$1"); mkdir -p "$out"
R=$PWD; T=$(mktemp -d); img=$T/img
mkdir -p $img/opt/tk8s/bin $img/opt/tk8s/lib $img/opt/rocm $img/bin
cp $R/tritonk8ssupervisor_amd/bin/tk8s-gpuinfo $img/opt/tk8s/bin/
cp $R/tritonk8ssupervisor_amd/lib/libtk8s.so $img/opt/tk8s/lib/
for b in /bin/sh; do cp -L $b $img/bin/; done
for l in $( (ldd $R/tritonk8ssupervisor_amd/bin/tk8s-gpuinfo; ldd /bin/sh; ldd /opt/rocm/lib/libamd_comgr.so.3) | awk '{for(i=1;i<=NF;i++) if ($i ~ /^\/(lib|usr)/) print $i}' | sort -u); do
  mkdir -p $img$(dirname $l); cp -L $l $img$l; done
ROCM=$(realpath /opt/rocm)
run() { sleep 1; timeout -k 5 60 "$@"; }  # 1 s apart: a GPU process's KFD release takes 0.1-0.2 s
run $R/tritonk8ssupervisor_amd/bin/tk8s-gpuinfo --no-links > $out/host.json 2> $out/host.err; echo "host rc=$?" > $out/status
minor=$(ls /dev/dri | grep -o 'renderD[0-9]*' | head -1 | tr -dc 0-9)
TK8S_PTRACE_LOG=$out/nojail.log run $R/tritonk8ssupervisor_amd/bin/tk8s-container --mode ptrace --rootfs $img \
  --upper $T/up1 --workdir / --bind-ro $ROCM:/opt/rocm --no-gpu-jail -- /bin/sh -c \
  'LD_LIBRARY_PATH=/opt/tk8s/lib:/opt/rocm/lib exec /opt/tk8s/bin/tk8s-gpuinfo --no-links' > $out/nojail.json 2> $out/nojail.err
echo "nojail rc=$?" >> $out/status
TK8S_PTRACE_LOG=$out/jail.log run $R/tritonk8ssupervisor_amd/bin/tk8s-container --mode ptrace --rootfs $img \
  --upper $T/up2 --workdir / --bind-ro $ROCM:/opt/rocm --allow-render $minor -- /bin/sh -c \
  'LD_LIBRARY_PATH=/opt/tk8s/lib:/opt/rocm/lib exec /opt/tk8s/bin/tk8s-gpuinfo --no-links' > $out/jail.json 2> $out/jail.err
echo "jail rc=$? minor=$minor" >> $out/status
for i in 1 2 3; do  # unlogged: the supervisor's own cost
  run $R/tritonk8ssupervisor_amd/bin/tk8s-container --mode ptrace --rootfs $img --upper $T/up3 --workdir / \
    --bind-ro $ROCM:/opt/rocm --allow-render $minor -- /bin/sh -c \
    'LD_LIBRARY_PATH=/opt/tk8s/lib:/opt/rocm/lib exec /opt/tk8s/bin/tk8s-gpuinfo --no-links' > $out/jail_nolog_$i.json 2>/dev/null
  run $R/tritonk8ssupervisor_amd/bin/tk8s-gpuinfo --no-links > $out/host_$i.json 2>/dev/null
done
ls -la /dev/dri /dev/kfd > $out/devs.txt 2>&1
rm -rf $T
