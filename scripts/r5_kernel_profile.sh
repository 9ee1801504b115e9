#!/usr/bin/env bash
# The burn-in payload's kernels on the final tree: per-kernel time (--kernel-trace --stats) for
# the HSA payload (the bring-up's default) and the HIP probe, then two counter passes (HBM bytes
# fetched, written) of the HSA payload, each in a run of its own.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5_kernels
mkdir -p $O
A="--all-devices --hbm-bytes 1073741824 --md5-bytes 268435456 --iters 5"
TK8S_PROBE_CLEAN_EXIT=1 timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/hsa -o run -- $R/tritonk8ssupervisor_amd/bin/tk8s-hsaprobe $A --out $O/hsa.json > $O/hsa.log 2>&1 &&
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/hip -o run -- $R/tritonk8ssupervisor_amd/bin/tk8s-probe $A --out $O/hip.json > $O/hip.log 2>&1 &&
TK8S_PROBE_CLEAN_EXIT=1 timeout -s KILL 60 rocprofv3 --kernel-trace --output-format csv --pmc FETCH_SIZE SQ_WAVES -d $O/pmc_fetch -o run -- $R/tritonk8ssupervisor_amd/bin/tk8s-hsaprobe $A --out $O/pmc_fetch.json > $O/pmc_fetch.log 2>&1 &&
TK8S_PROBE_CLEAN_EXIT=1 timeout -s KILL 60 rocprofv3 --kernel-trace --output-format csv --pmc WRITE_SIZE GRBM_GUI_ACTIVE -d $O/pmc_write -o run -- $R/tritonk8ssupervisor_amd/bin/tk8s-hsaprobe $A --out $O/pmc_write.json > $O/pmc_write.log 2>&1
