#!/usr/bin/env bash
# Code-object load time on the MI355X: RCCL's gfx950 code object vs synthetic 10/500-kernel ones.
set -o pipefail
out=gpurun_out/r5_coload
mkdir -p $out /tmp/coload
timeout -k 10 600 python3 -c "from tritonk8ssupervisor_amd.utils.build_native import build; build()" > $out/build.log 2>&1
timeout -k 10 120 python3 - <<'PY'
from tritonk8ssupervisor_amd.utils.rccl_unpack import OUT, LIB_NAME, elf_section
off, size = elf_section(str(OUT / LIB_NAME), ".hip_fatbin")[:2]
with open(OUT / LIB_NAME, "rb") as f:
    f.seek(off)
    open("/tmp/coload/fatbin.bin", "wb").write(f.read(size))
PY
/opt/rocm/lib/llvm/bin/clang-offload-bundler --unbundle --type=o --input=/tmp/coload/fatbin.bin \
  --targets=hipv4-amdgcn-amd-amdhsa--gfx950 --output=/tmp/coload/rccl_gfx950.co
for order in "build/k10.co build/k500.co /tmp/coload/rccl_gfx950.co"; do
  timeout -k 10 120 ./build/coload_bench - $order >> $out/results.jsonl
done
for f in /tmp/coload/rccl_gfx950.co; do
  COLOAD_SAMPLE=real timeout -k 10 120 ./build/coload_bench - $f >> $out/sampled.jsonl
done
cat $out/results.jsonl; head -c 6000 $out/sampled.jsonl
