"""Stand-ins for standard-library modules a daemon imports only through another module's import
statements and may never use: the real module loads on the first attribute the stand-in does not
carry itself.

The control plane imports ``asyncio``, which imports ``logging`` (a logger for its debug and
error messages), ``concurrent.futures`` (thread pools and cross-thread futures, which the
control plane never uses) and ``inspect`` (debug reprs, and checks on error paths and on
awaitables that are not coroutines). Together they are about 40 % of ``asyncio``'s import, and the
control plane's start is on the bring-up's critical path (controlplane/__main__.py). asyncio only
needs a few constants of them at import time; those are given here, and anything else -- an
error asyncio logs, a ``run_in_executor`` -- loads the real module then and is answered by it.
"""
from __future__ import annotations

import sys
import types


class _LazyModule(types.ModuleType):
    def __init__(self, name: str, attrs: dict):
        super().__init__(name)
        self.__dict__.update(attrs)
        self._lazy_real = None

    def __getattr__(self, attr):  # only for what the stand-in does not carry
        if attr.startswith("__") and attr.endswith("__"):
            raise AttributeError(attr)
        real = self.__dict__.get("_lazy_real")
        if real is None:
            if sys.modules.get(self.__name__) is self:
                del sys.modules[self.__name__]
            __import__(self.__name__)
            real = sys.modules[self.__name__]
            self.__dict__["_lazy_real"] = real
        return getattr(real, attr)


class _LazyLogger:
    """What ``logging.getLogger(name)`` returns from the stand-in: the real logger, once used."""

    def __init__(self, module: _LazyModule, name: str | None):
        self._module, self._name = module, name

    def __getattr__(self, attr):
        return getattr(self._module.getLogger_real(self._name), attr)


def install() -> None:
    """Stand in for ``logging``, ``inspect`` and ``concurrent.futures`` unless imported already."""
    if "logging" not in sys.modules:
        log = _LazyModule("logging", {"CRITICAL": 50, "FATAL": 50, "ERROR": 40, "WARNING": 30, "WARN": 30,
                                      "INFO": 20, "DEBUG": 10, "NOTSET": 0})
        log.getLogger = lambda name=None, _m=log: _LazyLogger(_m, name)
        log.getLogger_real = lambda name=None, _m=log: _m.__getattr__("getLogger")(name)
        sys.modules["logging"] = log
    if "inspect" not in sys.modules:
        sys.modules["inspect"] = _LazyModule("inspect", {})
    if "concurrent.futures" not in sys.modules:
        import concurrent  # the (empty) package itself is cheap

        cf = _LazyModule("concurrent.futures", {"FIRST_COMPLETED": "FIRST_COMPLETED",
                                                 "FIRST_EXCEPTION": "FIRST_EXCEPTION",
                                                 "ALL_COMPLETED": "ALL_COMPLETED"})
        sys.modules["concurrent.futures"] = cf
        concurrent.futures = cf
