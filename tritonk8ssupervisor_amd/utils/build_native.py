"""In-tree build of the tk8s native layer for gfx950 (MI355X).

Outputs (all in-tree so they travel to the GPU box with the repo snapshot):

* ``tritonk8ssupervisor_amd/lib/libtk8s.so`` — HIP kernels (N4-N7) and probes (N1); links only
  ``libamdhip64``.
* ``tritonk8ssupervisor_amd/lib/libtk8s_rccl.so`` — the RCCL validator (N3); the only artefact
  that links ``librccl`` (573 MB on ROCm 7.2), so the probe and gpuinfo payloads on the
  bring-up's critical path never map it.
* ``tritonk8ssupervisor_amd/_tk8s_native*.so`` — pybind11 module over both libraries.
* ``tritonk8ssupervisor_amd/_tk8s_topo*.so`` — pybind11 module of the CPU-only xGMI-aware
  allocator (N2 core); no HIP dependency so the node agent can load it safely.
* ``tritonk8ssupervisor_amd/bin/tk8s-{gpuinfo,probe,rccl}`` — the validation pod payloads.
* ``tritonk8ssupervisor_amd/bin/tk8s-smi`` — AMD SMI health/telemetry (links ``libamd_smi`` only,
  no HIP), run periodically by the node agent.

The reference has no native code at all; this build replaces nothing there.
Incremental: an output is rebuilt when any of its inputs or any header is newer.
"""
from __future__ import annotations

import concurrent.futures as cf
import json
import os
import shutil
import subprocess
import sys
import sysconfig
from pathlib import Path

REPO = Path(__file__).resolve().parents[2]
PKG = REPO / "tritonk8ssupervisor_amd"
NATIVE = REPO / "native"
OBJ = REPO / "build" / "native"
LIBDIR = PKG / "lib"
BINDIR = PKG / "bin"
ROCM = Path(os.environ.get("ROCM_PATH", "/opt/rocm"))
ARCH = os.environ.get("PYTORCH_ROCM_ARCH", "gfx950")

HIPCC = str(ROCM / "bin" / "hipcc")
CXX = shutil.which("g++") or "c++"

COMMON = ["-O3", "-std=c++17", "-fPIC", f"-I{NATIVE / 'include'}", "-Wall", "-Wno-unused-result"]
HIP_FLAGS = COMMON + [f"--offload-arch={ARCH}", "-munsafe-fp-atomics"]

LIB_SOURCES = [
    "src/stream_kernels.hip",
    "src/md5_kernels.hip",
    "src/probes.cpp",
]
RCCL_SOURCES = ["src/rccl_bench.cpp"]
# tools that need RCCL; every other tool links libtk8s.so only
RCCL_TOOLS = {"tk8s-rccl"}
TOOLS = {
    "tk8s-gpuinfo": "tools/tk8s_gpuinfo.cpp",
    "tk8s-probe": "tools/tk8s_probe.cpp",
    "tk8s-rccl": "tools/tk8s_rccl.cpp",
}


def ext_suffix() -> str:
    return sysconfig.get_config_var("EXT_SUFFIX") or ".so"


def native_module_path() -> Path:
    return PKG / f"_tk8s_native{ext_suffix()}"


def topo_module_path() -> Path:
    return PKG / f"_tk8s_topo{ext_suffix()}"


def lib_path() -> Path:
    return LIBDIR / "libtk8s.so"


def rccl_lib_path() -> Path:
    return LIBDIR / "libtk8s_rccl.so"


def _obj(rel: str) -> Path:
    src = Path(rel)
    return OBJ / (src.stem + src.suffix.replace(".", "_") + ".o")


def tool_path(name: str) -> Path:
    return BINDIR / name


def _headers() -> list[Path]:
    return sorted((NATIVE / "include").rglob("*.h")) + sorted((NATIVE / "tools").glob("*.h"))


def _stale(out: Path, inputs: list[Path]) -> bool:
    if not out.exists():
        return True
    t = out.stat().st_mtime
    return any(p.stat().st_mtime > t for p in inputs + _headers())


def _run(cmd: list[str], verbose: bool) -> None:
    """Run one compiler/linker command. Its ``-o`` output is written beside the target and renamed
    over it: a process executing or mapping the old file (a test, a running bring-up) never sees a
    half-written one."""
    out = cmd[cmd.index("-o") + 1] if "-o" in cmd[:-1] else None
    tmp = f"{out}.tmp{os.getpid()}" if out else None
    if tmp:
        cmd = list(cmd)
        cmd[cmd.index("-o") + 1] = tmp
    if verbose:
        print("+", " ".join(cmd), flush=True)
    res = subprocess.run(cmd, capture_output=True, text=True)
    if res.returncode != 0:
        if tmp and os.path.exists(tmp):
            os.unlink(tmp)
        raise RuntimeError(f"native build failed: {' '.join(cmd)}\n{res.stdout}\n{res.stderr}")
    if tmp:
        os.replace(tmp, out)


def _pybind_includes() -> list[str]:
    import pybind11  # noqa: PLC0415 (build-time only)

    return [f"-I{pybind11.get_include()}", f"-I{sysconfig.get_paths()['include']}"]


def build(force: bool = False, jobs: int | None = None, verbose: bool = False) -> dict:
    """Compile everything; returns {name: path} of the produced artefacts."""
    OBJ.mkdir(parents=True, exist_ok=True)
    LIBDIR.mkdir(parents=True, exist_ok=True)
    BINDIR.mkdir(parents=True, exist_ok=True)
    jobs = jobs or min(8, os.cpu_count() or 4)

    # 1. objects of libtk8s.so (hipcc, gfx950 device code)
    objs: list[tuple[Path, list[str]]] = []
    for rel in LIB_SOURCES + RCCL_SOURCES:
        src = NATIVE / rel
        obj = _obj(rel)
        if force or _stale(obj, [src]):
            objs.append((obj, [HIPCC, *HIP_FLAGS, "-c", str(src), "-o", str(obj)]))
    # tool objects and module objects compile in the same pool
    tool_objs = {}
    for name, rel in TOOLS.items():
        src = NATIVE / rel
        obj = OBJ / (src.stem + ".o")
        tool_objs[name] = obj
        if force or _stale(obj, [src]):
            objs.append((obj, [HIPCC, *COMMON, f"--offload-arch={ARCH}", "-c", str(src), "-o", str(obj)]))
    py_inc = _pybind_includes()
    nat_obj = OBJ / "native_module.o"
    nat_src = NATIVE / "bindings" / "native_module.cpp"
    if force or _stale(nat_obj, [nat_src]):
        objs.append((nat_obj, [HIPCC, *COMMON, f"--offload-arch={ARCH}", *py_inc, "-fvisibility=hidden", "-c",
                               str(nat_src), "-o", str(nat_obj)]))
    topo_srcs = [NATIVE / "src" / "topology.cpp", NATIVE / "bindings" / "topo_module.cpp"]
    topo_objs = [OBJ / (s.stem + "_topo.o") for s in topo_srcs]
    for s, o in zip(topo_srcs, topo_objs):
        if force or _stale(o, [s]):
            objs.append((o, [CXX, *COMMON, *py_inc, "-fvisibility=hidden", "-c", str(s), "-o", str(o)]))

    with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
        list(ex.map(lambda oc: _run(oc[1], verbose), objs))

    lib_objs = [_obj(r) for r in LIB_SOURCES]
    rccl_objs = [_obj(r) for r in RCCL_SOURCES]
    hip_libs = [f"-L{ROCM / 'lib'}", "-lamdhip64", f"-Wl,-rpath,{ROCM / 'lib'}"]
    lib = lib_path()
    if force or _stale(lib, lib_objs):
        _run([HIPCC, "-shared", "-fPIC", f"--offload-arch={ARCH}", *[str(o) for o in lib_objs],
              "-o", str(lib), *hip_libs], verbose)
    rlib = rccl_lib_path()
    if force or _stale(rlib, rccl_objs + [lib]):
        _run([HIPCC, "-shared", "-fPIC", *[str(o) for o in rccl_objs], "-o", str(rlib),
              f"-L{LIBDIR}", "-ltk8s", "-Wl,-rpath,$ORIGIN", *hip_libs, "-lrccl"], verbose)

    links = []
    nat = native_module_path()
    if force or _stale(nat, [nat_obj, lib, rlib]):
        links.append([HIPCC, "-shared", "-fPIC", str(nat_obj), "-o", str(nat), f"-L{LIBDIR}",
                      "-ltk8s_rccl", "-ltk8s", "-Wl,-rpath,$ORIGIN/lib", *hip_libs, "-lrccl"])
    topo = topo_module_path()
    if force or _stale(topo, topo_objs):
        links.append([CXX, "-shared", "-fPIC", *[str(o) for o in topo_objs], "-o", str(topo)])
    for name, obj in tool_objs.items():
        out = tool_path(name)
        rccl = ["-ltk8s_rccl"] if name in RCCL_TOOLS else []
        deps = [obj, lib] + ([rlib] if rccl else [])
        if force or _stale(out, deps):
            links.append([HIPCC, str(obj), "-o", str(out), f"-L{LIBDIR}", *rccl, "-ltk8s",
                          "-Wl,-rpath,$ORIGIN/../lib", *hip_libs, *(["-lrccl"] if rccl else []),
                          "-Wl,--export-dynamic-symbol=opendir", "-ldl", "-lpthread"])  # cachewalk.h
    with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
        list(ex.map(lambda c: _run(c, verbose), links))

    smi_srcs = [NATIVE / "src" / "smi_health.cpp", NATIVE / "tools" / "tk8s_smi.cpp"]
    smi = tool_path("tk8s-smi")
    if force or _stale(smi, smi_srcs):
        _run([CXX, "-O2", "-std=c++17", "-Wall", f"-I{NATIVE / 'include'}", f"-I{ROCM / 'include'}",
              *[str(x) for x in smi_srcs], "-o", str(smi), f"-L{ROCM / 'lib'}", "-lamd_smi",
              f"-Wl,-rpath,{ROCM / 'lib'}"], verbose)

    # The host-only tools every pod start execs (the validation payload's tk8s-reuse, the jail, the
    # container runtime, the restart supervisor) carry their C++ runtime: no libstdc++ to map and
    # relocate -- ~0.7 ms off each exec on the bring-up's critical path (libc stays shared).
    static = ["-static-libstdc++", "-static-libgcc"]
    reuse_src = NATIVE / "tools" / "tk8s_reuse.cpp"
    reuse_bin = tool_path("tk8s-reuse")
    if force or _stale(reuse_bin, [reuse_src, Path(__file__)]):
        _run([CXX, "-O2", "-std=c++17", "-Wall", *static, str(reuse_src), "-o", str(reuse_bin)], verbose)

    # pod isolation: the GPU jail (process pods) and the container runtime (image pods), no HIP
    jail_hdr = NATIVE / "tools" / "gpujail.h"
    for tname, tsrc in (("tk8s-gpujail", "tk8s_gpujail.cpp"), ("tk8s-container", "tk8s_container.cpp")):
        src = NATIVE / "tools" / tsrc
        if force or _stale(tool_path(tname), [src, jail_hdr, NATIVE / "tools" / "ptrace_root.h", Path(__file__)]):
            _run([CXX, "-O2", "-std=c++17", "-Wall", "-Wextra", *static, str(src), "-o", str(tool_path(tname))],
                 verbose)
    jail = tool_path("tk8s-gpujail")

    sup_src = NATIVE / "tools" / "tk8s_supervise.cpp"
    sup = tool_path("tk8s-supervise")
    if force or _stale(sup, [sup_src, Path(__file__)]):
        _run([CXX, "-O2", "-std=c++17", "-Wall", *static, str(sup_src), "-o", str(sup)], verbose)

    # Device-only code objects of the validation kernels (the same sources as libtk8s.so) for
    # tk8s-hsaprobe, which dispatches them on ROCr directly, and that tool itself (no HIP).
    cos = {}
    for rel, name in (("src/stream_kernels.hip", "tk8s_stream.co"), ("src/md5_kernels.hip", "tk8s_md5.co")):
        co = LIBDIR / name
        cos[name] = co
        if force or _stale(co, [NATIVE / rel]):
            _run([HIPCC, *HIP_FLAGS, "--cuda-device-only", "--no-gpu-bundle-output", "-c", str(NATIVE / rel),
                  "-o", str(co)], verbose)
    hsa_src = NATIVE / "tools" / "tk8s_hsaprobe.cpp"
    hsa_bin = tool_path("tk8s-hsaprobe")
    if force or _stale(hsa_bin, [hsa_src]):
        _run([CXX, "-O2", "-std=c++17", "-Wall", f"-I{NATIVE / 'include'}", f"-I{NATIVE / 'tools'}",
              f"-I{ROCM / 'include'}", str(hsa_src), "-o", str(hsa_bin), f"-L{ROCM / 'lib'}", "-lhsa-runtime64",
              f"-Wl,-rpath,{ROCM / 'lib'}", "-Wl,--export-dynamic-symbol=opendir", "-ldl", "-lpthread"], verbose)  # cachewalk.h

    precompile_python()
    from .rccl_unpack import unpack

    try:  # RCCL's gfx950 device code unpacked once per host (the fabric check's communicator start)
        rccl_unpacked = unpack(verbose=verbose)
    except Exception as e:  # noqa: BLE001 - an optional speed-up: the installed library stays usable
        rccl_unpacked = {"ok": False, "why": str(e)}
    out = {"libtk8s": lib, "libtk8s_rccl": rlib, "native_module": nat, "topo_module": topo, "tk8s-supervise": sup,
           "tk8s-gpujail": jail, "tk8s-container": tool_path("tk8s-container"),
           "tk8s-smi": smi, "tk8s-reuse": reuse_bin, "tk8s-hsaprobe": hsa_bin, **cos,
           "rccl-unpacked": rccl_unpacked.get("path") or f"no ({rccl_unpacked.get('why')})"}
    out.update({n: tool_path(n) for n in TOOLS})
    return out


# what the CLI, the control plane and the agents import: warmed into the byte-code cache by
# precompile_python, evicted from the page cache by bench.py --cold-evict
BRINGUP_MODULES = [
    "tritonk8ssupervisor_amd.cli.main", "tritonk8ssupervisor_amd.cli.kubectl", "tritonk8ssupervisor_amd.orchestrator",
    "tritonk8ssupervisor_amd.playbook", "tritonk8ssupervisor_amd.playbook_modules", "tritonk8ssupervisor_amd.kube",
    "tritonk8ssupervisor_amd.wizard", "tritonk8ssupervisor_amd.controlplane.server", "tritonk8ssupervisor_amd.burnin",
    "tritonk8ssupervisor_amd.agent.agent", "tritonk8ssupervisor_amd.ops.fakeprobe", "yaml", "argparse", "asyncio",
    "tritonk8ssupervisor_amd.controlplane.client", "tritonk8ssupervisor_amd.controlplane.ingress",
    "tritonk8ssupervisor_amd.controlplane.dns", "tritonk8ssupervisor_amd.utils.k8senv",
    "tritonk8ssupervisor_amd.earlyburn", "tritonk8ssupervisor_amd.provider.hostreg",
    "tritonk8ssupervisor_amd.parallel.dist_allreduce"]


def precompile_python() -> None:
    """Byte-compile the package with source-HASH-checked .pyc files.

    Every bring-up starts the CLI, the control plane and one agent per worker as fresh
    interpreters; without a valid .pyc each compiles its modules from source (measured 54 ms
    of the CLI's start-up on the GPU box, where the snapshot's file mtimes do not match the
    timestamp-based .pyc files and the tree may not be writable by the daemons' user).
    Hash-checked .pyc files stay valid across copies and mtime changes and are rebuilt here
    when a source file changes.
    """
    import compileall
    import py_compile

    prefix = sys.pycache_prefix
    sys.pycache_prefix = None  # the in-package __pycache__ copies, for interpreters without the prefix
    try:
        compileall.compile_dir(str(PKG), quiet=2, workers=1, force=True,
                               invalidation_mode=py_compile.PycInvalidationMode.CHECKED_HASH)
    finally:
        sys.pycache_prefix = prefix
    # Warm the shared prefix cache (tritonk8ssupervisor_amd/__init__.py) with everything the CLI,
    # the control plane and the agents import, stdlib and PyYAML included.
    env = dict(os.environ)
    env["PYTHONPATH"] = os.pathsep.join([str(REPO)] + [p for p in env.get("PYTHONPATH", "").split(os.pathsep) if p])
    mods = BRINGUP_MODULES
    code = "import importlib\nfor m in %r:\n    importlib.import_module(m)\n" % (mods[:-1] + ["tritonk8ssupervisor_amd.provision"],)
    for flag in (["-S"], []):
        subprocess.run([sys.executable, *flag, "-c", code], env=env, cwd=str(REPO), capture_output=True, timeout=120)


def _probe_libraries() -> list[str]:
    """The shared libraries the GPU burn-in (tk8s-hsaprobe) maps, as the dynamic loader resolves them."""
    try:
        out = subprocess.run(["ldd", str(tool_path("tk8s-hsaprobe"))], capture_output=True, text=True, timeout=10).stdout
    except (OSError, subprocess.SubprocessError):
        return []
    return [parts[1].split("(")[0].strip() for parts in (line.split("=>") for line in out.splitlines())
            if len(parts) == 2 and parts[1].strip().startswith("/")]


def bringup_files(env: dict | None = None, relative: bool = True) -> list[str]:
    """Every file a bring-up's processes read from disk, in about the order they read them: the
    interpreter and its shared library, the stdlib and third-party modules the CLI, the control
    plane and the agents import (asked of a child interpreter: import order), the tk8s package,
    its playbook / manifest / Terraform files and native tools, the shared libraries the GPU
    burn-in maps (bench.py --cold-evict). Paths under the tree are relative to it (``relative``)."""
    import sysconfig

    code = ("import importlib, json, sys\nfor m in %r:\n    importlib.import_module(m)\n"
            "print(json.dumps([getattr(m, '__file__', None) or '' for m in list(sys.modules.values())]))"
            % (BRINGUP_MODULES,))
    files: list[str] = [os.path.realpath(sys.executable)]
    lib = sysconfig.get_config_var("INSTSONAME")
    if lib:
        files.append(os.path.join(sysconfig.get_config_var("LIBDIR") or "/usr/lib", lib))
    try:
        out = subprocess.run([sys.executable, "-S", "-c", code], env=env, cwd=str(REPO), capture_output=True,
                             text=True, timeout=120)
        files += [f for f in json.loads(out.stdout.strip().splitlines()[-1]) if f]
    except (OSError, ValueError, IndexError, subprocess.SubprocessError):
        pass
    for sub in ("tritonk8ssupervisor_amd", "ansible", "terraform", "manifests"):
        for dirpath, dirnames, names in os.walk(REPO / sub):
            dirnames[:] = sorted(d for d in dirnames if d != "__pycache__")
            files += [os.path.join(dirpath, f) for f in sorted(names)]
    files += _probe_libraries()
    out_list, seen = [], set()
    for f in files:
        real = os.path.realpath(f)
        if real in seen or not os.path.isfile(real):
            continue
        seen.add(real)
        rel = os.path.relpath(real, REPO)
        out_list.append(rel if relative and not rel.startswith("..") else real)
    return out_list


def main(argv: list[str] | None = None) -> int:
    argv = sys.argv[1:] if argv is None else argv
    res = build(force="--force" in argv, verbose="-v" in argv)
    for k, v in res.items():
        print(f"{k}: {v}")
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
