set -e
mkdir -p gpurun_out/hsat2
B=tritonk8ssupervisor_amd/bin/tk8s-hsaprobe
A="--all-devices --gpuinfo --hbm-bytes 1073741824 --md5-bytes 268435456 --iters 3"
for i in 1 2 3 4 5 6; do
  timeout -k 5 60 $B $A --out gpurun_out/hsat2/par$i.json > /dev/null; sleep 1
  TK8S_HSAPROBE_SERIAL_SETUP=1 timeout -k 5 60 $B $A --out gpurun_out/hsat2/ser$i.json > /dev/null; sleep 1
done
LD_DEBUG=statistics timeout -k 5 60 $B $A --out gpurun_out/hsat2/ld.json > /dev/null 2> gpurun_out/hsat2/ld_stats.txt
echo done
