#!/usr/bin/env bash
# Where HIP's runtime start goes (the multi-GPU burn-in runs the HIP probe, tk8s-probe): a 1 ms
# wall-clock sample of hipInit + hipSetDevice + hipFree, then tk8s-probe's runtime start with
# and without glibc's huge-page malloc, interleaved, 4 rounds.
set -o pipefail
out=gpurun_out/r5_hipinit
mkdir -p $out
for v in base thp; do
  if [[ $v == thp ]]; then export GLIBC_TUNABLES=glibc.malloc.hugetlb=1; else unset GLIBC_TUNABLES; fi
  COLOAD_SAMPLE=real timeout -k 10 60 ./build/coload_bench - build/k10.co > $out/sampled_$v.jsonl
done
for r in 1 2 3 4; do
  for v in base thp; do
    if [[ $v == thp ]]; then export GLIBC_TUNABLES=glibc.malloc.hugetlb=1; else unset GLIBC_TUNABLES; fi
    timeout -k 10 60 ./tritonk8ssupervisor_amd/bin/tk8s-probe --hbm-bytes 268435456 --md5-bytes 16777216 \
      --copy-bytes 16777216 --iters 2 > $out/probe.json
    echo "$v $(python3 -c 'import json,sys; d=json.load(open(sys.argv[1])); print(d.get("ok"), json.dumps(d.get("timings_ms")))' $out/probe.json)" >> $out/probe.txt
  done
done
unset GLIBC_TUNABLES
cat $out/probe.txt
