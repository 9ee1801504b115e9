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


# optional modules the stdlib probes for on Linux (subprocess: msvcrt, _winapi; ntpath: nt, ...;
# copy and pickle: Jython's org.python.core -- an "org" namespace package in site-packages made
# that probe load `site` and three packages, ~2.6 ms of the first `import copy`)
_PLATFORM_PROBES = frozenset({"msvcrt", "_winapi", "nt", "winreg", "_winreg", "_overlapped", "_scproxy", "vms_lib",
                              "java", "_wmi", "org"})


def _fast_site() -> None:
    """Our daemons and the CLI start with ``python3 -S`` (no ``site`` processing: ~30 ms less
    per interpreter on the bring-up's critical path, where three start one after another).
    Third-party packages (PyYAML, jinja2, grpc) must stay importable, so the site-packages
    directories are appended -- without executing their ``.pth`` hooks -- but only when an import
    first needs them: a finder placed last on ``sys.meta_path`` sees only imports nothing else
    could satisfy, and when the module is in one of those directories it adds them all (once) and
    returns its spec. A bring-up whose caches are warm never loads a third-party package."""
    import sys

    if not sys.flags.no_site or any(getattr(f, "_tk8s_late_site", False) for f in sys.meta_path):
        return

    class _LateSite:
        _tk8s_late_site = True

        @classmethod
        def find_spec(cls, name, path=None, target=None):
            if path is not None or name in _PLATFORM_PROBES:  # a submodule, or the stdlib probing
                return None                                       # for another OS: nothing to add
            import site
            from importlib.machinery import PathFinder

            dirs = [d for d in site.getsitepackages() + [site.getusersitepackages()] if d not in sys.path]
            spec = PathFinder.find_spec(name, dirs)
            if spec is not None:  # a third-party package: from now on the directories are on sys.path
                sys.meta_path.remove(cls)
                sys.path.extend(dirs)
            return spec  # None: a probe for an optional module (ntpath's _winapi, ...) stays a miss

    sys.meta_path.append(_LateSite)


def _pycache_prefix() -> None:
    """Keep byte code in a writable in-tree cache (``build/pycache``) for every interpreter of a
    bring-up and its children. On the GPU hosts the daemons' user cannot write the system
    ``__pycache__`` dirs and part of the stdlib and site-packages ships without valid .pyc
    files: measured there, each interpreter start compiled 66 modules from source (~50 ms),
    three times on the critical path. ``build()`` warms this cache once."""
    import os
    import sys

    if sys.pycache_prefix or os.environ.get("PYTHONPYCACHEPREFIX") or os.environ.get("TK8S_NO_PYCACHE_PREFIX"):
        return
    d = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "build", "pycache")
    try:
        os.makedirs(d, exist_ok=True)
    except OSError:
        return
    if os.access(d, os.W_OK):
        sys.pycache_prefix = d
        os.environ["PYTHONPYCACHEPREFIX"] = d


# TK8S_SHORTCUTS=0: every start-up shortcut of docs/architecture.md ("Start-up shortcuts and their
# off-switches") off at once, the bring-up's plain path. setup.sh sets the same switches for the
# ones it acts on before Python starts; bench.py reports this path as plain_path_s.
SHORTCUT_SWITCHES = {
    "TK8S_HOST_BURNIN": "0",          # the early host burn-in (earlyburn.py)
    "TK8S_CP_ZYGOTE": "0",            # the control-plane zygote
    "TK8S_AGENT_ZYGOTE": "0",         # the node-agent zygotes
    "TK8S_HSA_CPU_CACHES": "1",       # ROCr's per-CPU cache walk runs as usual
    "TK8S_YAML_CACHE": "off",         # the parse caches
    "TK8S_NO_PYCACHE_PREFIX": "1",    # the shared byte-code prefix
    "TK8S_PLAY_INLINE": "0",          # inline file-only tasks
    "TK8S_INPROCESS_BOOTSTRAP": "0",  # the in-process machine bootstrap
    "TK8S_FAST_ARGS": "0",            # the hand-written argument parsers (argparse instead)
    "TK8S_SKIP_SITE": "0",            # daemons' interpreters start without -S (utils/procs.plain_argv)
    "TK8S_RCCL_UNPACKED": "0",        # the fabric Job's RCCL with its device code unpacked (utils/rccl_unpack.py)
    "TK8S_RCCL_THP": "0",             # the fabric Job's malloc on transparent huge pages (fabric.py)
    "TK8S_RCCL_PREWARM": "0",         # the rank's RCCL code load and stream on threads (tk8s_rccl.cpp)
}


def _shortcuts_off() -> None:
    import os

    if os.environ.get("TK8S_SHORTCUTS", "1") == "0":
        os.environ.update(SHORTCUT_SWITCHES)


def shortcut_on(switch: str) -> bool:
    """Whether the shortcut behind ``switch`` (a key of SHORTCUT_SWITCHES) is on."""
    import os

    v = os.environ.get(switch)
    return v is None or v != SHORTCUT_SWITCHES[switch]


_shortcuts_off()
_fast_site()
_pycache_prefix()
