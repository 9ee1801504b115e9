# Follow-up of gpu_init_costs.sh: (1) does the device kernarg pool (HIP_FORCE_DEV_KERNARG) make a
# stream cost 20 ms? (2) does hsa_init get slower when the previous GPU process exited just
# before (deferred KFD teardown), i.e. does a gap between GPU processes make it fast again?
set -euo pipefail
cd "$GRAFT_REPO_ROOT"
o=gpurun_out/init_costs2
mkdir -p $o
/opt/rocm/bin/hipcc -O2 --offload-arch=gfx950 -o /tmp/init_costs native/bench/init_costs.hip
g++ -O2 -std=c++17 -I/opt/rocm/include native/bench/hsa_init_costs.cpp -L/opt/rocm/lib -lhsa-runtime64 -Wl,-rpath,/opt/rocm/lib -o /tmp/hsa_init_costs
for i in 1 2 3; do HIP_FORCE_DEV_KERNARG=0 timeout -k 5 60 /tmp/init_costs; done > $o/kernarg0.jsonl
for i in 1 2 3; do timeout -k 5 60 /tmp/init_costs; done > $o/plain.jsonl
for gap in 0 0 0 2 2 2 0 0 5 5; do sleep $gap; echo "{\"gap_s\": $gap, \"r\": $(timeout -k 5 60 /tmp/hsa_init_costs)}"; done > $o/hsa_gaps.jsonl
HIP_FORCE_DEV_KERNARG=0 AMD_LOG_LEVEL=4 timeout -k 5 60 /tmp/init_costs > $o/amd_log4_kernarg0.txt 2>&1
