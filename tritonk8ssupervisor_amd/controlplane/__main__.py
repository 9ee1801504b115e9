import sys

from .server import main

if len(sys.argv) == 3 and sys.argv[1] == "--await-args":
    # Zygote (earlyburn.controlplane_zygote): the imports above are done; the arguments -- the
    # master's address and port -- arrive once the master machine exists.
    from .server import await_args

    raise SystemExit(main(await_args(sys.argv[2])))

raise SystemExit(main())
