"""tritonk8ssupervisor_amd — MI355X-native cluster bring-up (control plane + GPU workers).

Same capabilities and public surface as cheapRoc/tritonK8ssupervisor (``./setup.sh`` wizard,
``./setup.sh -c`` teardown, ``terraform/{master,host}`` + ``ansible/clusterUp.yml`` layout), but
targeting one 8x AMD Instinct MI355X (gfx950) node: a local provider instead of Joyent Triton,
an in-repo control plane + node agents instead of Rancher 1.x, and a native HIP/RCCL validation
stack (device discovery, HBM/MD5/xGMI probes, RCCL all-reduce) that must pass before a GPU
worker counts as Ready. See SURVEY.md for the reference map.

Keep this module import-light: node agents and the control plane start as separate processes
and their start-up time is part of the bring-up metric.
"""

__version__ = "0.1.0"


def _fast_site() -> None:
    """Our daemons and the CLI start with ``python3 -S`` (no ``site`` processing: ~30 ms less
    per interpreter on the bring-up's critical path, where three start one after another).
    Append the site-packages directories ourselves -- without executing their ``.pth`` hooks --
    so third-party packages (PyYAML) stay importable."""
    import sys

    if not sys.flags.no_site:
        return
    import site

    for d in site.getsitepackages() + [site.getusersitepackages()]:
        if d not in sys.path:
            sys.path.append(d)


_fast_site()
