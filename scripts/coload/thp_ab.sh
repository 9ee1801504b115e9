#!/usr/bin/env bash
# RCCL's code-object load is ~190 ms of memcpy into freshly faulted 4 KiB pages (HIP's stream
# copy, comgr's set_data, ...; gpurun_out/r5_coload/sampled.jsonl). A/B: glibc's malloc on
# transparent huge pages (GLIBC_TUNABLES=glibc.malloc.hugetlb=1) for the load alone and for the
# fabric Job's tk8s-rccl communicator start. Interleaved, 4 rounds.
set -o pipefail
out=gpurun_out/r5_thp
mkdir -p $out /tmp/coload /tmp/thp
timeout -k 10 600 python3 -c "from tritonk8ssupervisor_amd.utils.build_native import build; build()" > $out/build.log 2>&1
{ cat /sys/kernel/mm/transparent_hugepage/enabled; cat /sys/kernel/mm/transparent_hugepage/defrag; ldd --version | head -1; } > $out/system.txt
lib=$(python3 -c "from tritonk8ssupervisor_amd.utils.rccl_unpack import library_dir; print(library_dir() or '')")
[[ -n "$lib" ]] || exit 3
if [[ ! -f /tmp/coload/rccl_gfx950.co ]]; then
  timeout -k 10 120 python3 - <<'PY'
from tritonk8ssupervisor_amd.utils.rccl_unpack import OUT, LIB_NAME, elf_section
off, size = elf_section(str(OUT / LIB_NAME), ".hip_fatbin")[:2]
with open(OUT / LIB_NAME, "rb") as f:
    f.seek(off)
    open("/tmp/coload/fatbin.bin", "wb").write(f.read(size))
PY
  /opt/rocm/lib/llvm/bin/clang-offload-bundler --unbundle --type=o --input=/tmp/coload/fatbin.bin \
    --targets=hipv4-amdgcn-amd-amdhsa--gfx950 --output=/tmp/coload/rccl_gfx950.co
fi
for r in 1 2 3 4; do
  for v in base thp; do
    if [[ $v == thp ]]; then export GLIBC_TUNABLES=glibc.malloc.hugetlb=1; else unset GLIBC_TUNABLES; fi
    echo "$v $(timeout -k 10 120 ./build/coload_bench - /tmp/coload/rccl_gfx950.co | tail -1)" >> $out/coload.txt
    LD_LIBRARY_PATH=$lib timeout -k 10 120 ./tritonk8ssupervisor_amd/bin/tk8s-rccl --group-index 0 --devices 0 --nranks 1 \
      --uid-file /tmp/thp/uid_${v}_$r --max-bytes 4194304 --iters 3 --warmup 1 > /tmp/thp/out.json 2>> $out/rccl.err
    echo "$v $(tail -1 /tmp/thp/out.json | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ok"], d.get("comm_init_ms"))')" >> $out/rccl.txt
  done
done
unset GLIBC_TUNABLES
cat $out/system.txt $out/coload.txt $out/rccl.txt
