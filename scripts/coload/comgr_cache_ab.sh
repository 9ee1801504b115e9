#!/usr/bin/env bash
# HIP's first stream on a device runs comgr (its blit kernels are compiled at run time): with and
# without comgr's own cache (AMD_COMGR_CACHE=1, AMD_COMGR_CACHE_DIR), interleaved, 4 rounds.
set -o pipefail
out=gpurun_out/r5_comgr_cache
mkdir -p $out
rm -rf /tmp/tk8s-comgr-cache
for r in 1 2 3 4; do
  for v in base cache; do
    sleep 1.5
    if [[ $v == base ]]; then res=$(timeout -k 10 60 ./build/hipdev_bench) || exit 1
    else res=$(AMD_COMGR_CACHE=1 AMD_COMGR_CACHE_DIR=/tmp/tk8s-comgr-cache timeout -k 10 60 ./build/hipdev_bench) || exit 1; fi
    echo "$v $res" >> $out/results.txt
  done
done
{ echo "defaults: AMD_COMGR_CACHE=${AMD_COMGR_CACHE-unset} XDG_CACHE_HOME=${XDG_CACHE_HOME-unset} HOME=$HOME"; ls -la $HOME/.cache 2>&1 | head; du -sh /tmp/tk8s-comgr-cache 2>&1; ls /tmp/tk8s-comgr-cache 2>&1 | head; } > $out/cache_state.txt
cat $out/results.txt $out/cache_state.txt
