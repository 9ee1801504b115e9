"""GPU ops of the tk8s validation stack (HIP kernels for gfx950, built in-tree).

``native()`` returns the pybind11 module ``_tk8s_native`` and raises loudly when it is missing:
there is no silent PyTorch fallback for a validation kernel.
"""
from __future__ import annotations

import importlib
import json
from pathlib import Path
from types import ModuleType

PKG = Path(__file__).resolve().parents[1]
BIN = PKG / "bin"


class NativeUnavailable(RuntimeError):
    """The in-tree native build is missing (run ``python -m tritonk8ssupervisor_amd.utils.build_native``)."""


def _load(name: str) -> ModuleType:
    try:
        return importlib.import_module(f"tritonk8ssupervisor_amd.{name}")
    except ImportError as e:  # pragma: no cover - exercised only without a build
        raise NativeUnavailable(
            f"tritonk8ssupervisor_amd.{name} is not built: run "
            "`python -m tritonk8ssupervisor_amd.utils.build_native` (or __graft_entry__.build())"
        ) from e


def native() -> ModuleType:
    """HIP kernels + probes + RCCL validator (loads libamdhip64; does not init the GPU)."""
    return _load("_tk8s_native")


def topo() -> ModuleType:
    """CPU-only topology allocator (no HIP dependency)."""
    return _load("_tk8s_topo")


def tool(name: str) -> Path:
    """Path of a native CLI tool (tk8s-gpuinfo, tk8s-probe, tk8s-rccl)."""
    p = BIN / name
    if not p.exists():
        raise NativeUnavailable(f"{p} is not built")
    return p


def gpuinfo(with_links: bool = True) -> dict:
    return json.loads(native().gpuinfo_json(with_links))
