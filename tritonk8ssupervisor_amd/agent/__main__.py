"""Node agent entry: ``python -S -c 'import tritonk8ssupervisor_amd.agent.__main__' ARGS``.

``--await-args FILE`` is the zygote form (earlyburn.agent_zygotes): the interpreter starts and
imports with the CLI, then waits for ``{"argv": [...], "env": {...}, "cwd": DIR}`` -- what the
worker's boot hook would have started the agent with -- applies the environment and directory,
and runs the agent with that argv.
"""
import sys

from .agent import main

if len(sys.argv) == 3 and sys.argv[1] == "--await-args":
    import os

    from ..utils.trace import trace
    from ..utils.zygote import await_json

    trace("agent", "zygote imported")
    spec = await_json(sys.argv[2])
    os.environ.update({str(k): str(v) for k, v in (spec.get("env") or {}).items()})
    if spec.get("cwd"):
        os.chdir(spec["cwd"])
    trace("agent", "zygote args received")
    raise SystemExit(main([str(a) for a in spec["argv"]]))

raise SystemExit(main())
