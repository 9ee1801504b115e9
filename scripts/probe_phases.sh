set -o pipefail
mkdir -p gpurun_out/r5_probe_phases
for i in 1 2 3; do
  sleep 1.5
  timeout -k 10 60 ./tritonk8ssupervisor_amd/bin/tk8s-hsaprobe --all-devices --gpuinfo --hbm-bytes 1073741824 --md5-bytes 268435456 --iters 3 --out gpurun_out/r5_probe_phases/hsa_$i.json > /dev/null
  sleep 1.5
  timeout -k 10 60 ./tritonk8ssupervisor_amd/bin/tk8s-probe --all-devices --gpuinfo --hbm-bytes 1073741824 --md5-bytes 268435456 --iters 3 --out gpurun_out/r5_probe_phases/hip_$i.json > /dev/null
done
