#!/usr/bin/env bash
# HIP device first-use costs (build/hipdev_bench) under ROCclr / ROCr knobs, interleaved, 3 rounds.
set -o pipefail
out=gpurun_out/r5_hipdev_env
mkdir -p $out
for r in 1 2 3; do
  for v in ${VARIANTS:-base HIP_FORCE_DEV_KERNARG=1 ROC_AQL_QUEUE_SIZE=4096 GPU_MAX_HW_QUEUES=1 HSA_ENABLE_SDMA=0}; do
    sleep 1.5
    if [[ $v == base ]]; then res=$(timeout -k 10 60 ./build/hipdev_bench) || exit 1
    else res=$(env $v timeout -k 10 60 ./build/hipdev_bench) || exit 1; fi
    echo "$v $res" >> $out/results.txt
  done
done
cat $out/results.txt
