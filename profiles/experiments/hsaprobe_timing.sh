set -e
mkdir -p gpurun_out/hsat
B=tritonk8ssupervisor_amd/bin/tk8s-hsaprobe
for i in 1 2 3 4 5; do
  t0=$(date +%s%N)
  timeout -k 5 60 $B --all-devices --gpuinfo --hbm-bytes 1073741824 --md5-bytes 268435456 --iters 3 --out gpurun_out/hsat/r$i.json > /dev/null
  t1=$(date +%s%N)
  echo "run $i wall_ms=$(( (t1-t0)/1000000 ))" >> gpurun_out/hsat/wall.txt
  sleep 1
done
