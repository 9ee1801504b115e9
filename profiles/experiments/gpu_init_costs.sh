set -euo pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/init_costs
/opt/rocm/bin/hipcc -O2 --offload-arch=gfx950 -o /tmp/init_costs native/bench/init_costs.hip
for i in 1 2 3 4; do timeout -k 5 60 /tmp/init_costs; done > gpurun_out/init_costs/plain.jsonl
for i in 1 2 3 4; do timeout -k 5 60 /tmp/init_costs null; done > gpurun_out/init_costs/null.jsonl
for i in 1 2 3; do ROCR_VISIBLE_DEVICES=0 timeout -k 5 60 /tmp/init_costs; done > gpurun_out/init_costs/rocr0.jsonl
for i in 1 2 3; do HSA_ENABLE_SDMA=0 timeout -k 5 60 /tmp/init_costs; done > gpurun_out/init_costs/nosdma.jsonl
ls /dev/dri/ > gpurun_out/init_costs/dri.txt; ls /sys/class/kfd/kfd/topology/nodes | wc -l >> gpurun_out/init_costs/dri.txt
nproc >> gpurun_out/init_costs/dri.txt
g++ -O2 -std=c++17 -I/opt/rocm/include native/bench/hsa_init_costs.cpp -L/opt/rocm/lib -lhsa-runtime64 -Wl,-rpath,/opt/rocm/lib -o /tmp/hsa_init_costs
for i in 1 2 3 4; do timeout -k 5 60 /tmp/hsa_init_costs; done > gpurun_out/init_costs/hsa.jsonl
AMD_LOG_LEVEL=4 timeout -k 5 60 /tmp/init_costs > gpurun_out/init_costs/amd_log4.txt 2>&1
