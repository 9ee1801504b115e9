"""Control plane entry: ``python -S -c 'import tritonk8ssupervisor_amd.controlplane.__main__' ARGS``
(``-c``, not ``-m``: runpy and importlib.util cost ~4 ms of the daemon's start on the MI355X host,
and the start is on the bring-up's critical path; ``sys.argv`` has the same positions either way).

The control plane serves plain HTTP only, so ``ssl`` is kept out: asyncio imports it when it can
(~4 ms, libssl included) and runs without it when the import fails. (Round 4 also stood in for
``logging`` / ``inspect`` / ``concurrent.futures`` until first use; round 5 measured it on the
MI355X -- headline medians 0.0649/0.0638 s with it, 0.0654/0.0637 s without,
profiles/r5_lazy_ab/ -- and removed it: the zygote imports them before its arguments arrive.)
"""
import sys

sys.modules.setdefault("ssl", None)  # type: ignore[arg-type]  -- `import ssl` -> ImportError

from .server import main  # noqa: E402

if len(sys.argv) == 3 and sys.argv[1] == "--await-args":
    # Zygote (earlyburn.controlplane_zygote): the imports above are done; the arguments -- the
    # master's address and port -- arrive once the master machine exists.
    from ..utils.trace import trace
    from .server import await_args

    trace("cp", "zygote imported")
    args = await_args(sys.argv[2])
    trace("cp", "zygote args received")
    raise SystemExit(main(args))

raise SystemExit(main())
