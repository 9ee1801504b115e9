"""A small thread pool (submit / map / as_completed) for the bring-up's fan-outs.

``concurrent.futures`` imports ``logging`` (and with it traceback, tokenize, string ...):
~2 ms on the MI355X host, ~7 ms on slow CPUs, on the critical path of every ``./setup.sh``.
Provisioning (one thread per machine) and the playbook engine (one per host and task) only
need what is here. Workers are daemon threads started on demand, so a pool a failed run never
shut down cannot keep the process alive.
"""
from __future__ import annotations

import threading
from collections import deque


class Future:
    __slots__ = ("_event", "_result", "_exc", "_callbacks", "_lock")

    def __init__(self):
        self._event = threading.Event()
        self._result = None
        self._exc: BaseException | None = None
        self._callbacks: list = []
        self._lock = threading.Lock()

    def _finish(self, result=None, exc: BaseException | None = None) -> None:
        with self._lock:
            self._result, self._exc = result, exc
            self._event.set()
            cbs, self._callbacks = self._callbacks, []
        for cb in cbs:
            cb(self)

    def add_done_callback(self, cb) -> None:
        with self._lock:
            if not self._event.is_set():
                self._callbacks.append(cb)
                return
        cb(self)

    def done(self) -> bool:
        return self._event.is_set()

    def result(self, timeout: float | None = None):
        if not self._event.wait(timeout):
            raise TimeoutError("future not done")
        if self._exc is not None:
            raise self._exc
        return self._result

    def exception(self, timeout: float | None = None) -> BaseException | None:
        if not self._event.wait(timeout):
            raise TimeoutError("future not done")
        return self._exc


class Pool:
    def __init__(self, max_workers: int, name: str = "pool"):
        self.max_workers = max(1, int(max_workers))
        self.name = name
        self._queue: deque = deque()
        self._cv = threading.Condition()
        self._threads: list[threading.Thread] = []
        self._idle = 0
        self._shutdown = False

    def submit(self, fn, *args, **kwargs) -> Future:
        fut = Future()
        with self._cv:
            if self._shutdown:
                raise RuntimeError("cannot submit to a pool that was shut down")
            self._queue.append((fut, fn, args, kwargs))
            if self._idle > 0:
                # claim one waiting worker now: counting it as idle until it has woken up would
                # let the next submit skip spawning while this worker is taken (a lost task when
                # every running task waits on a later one)
                self._idle -= 1
                self._cv.notify()
            elif len(self._threads) < self.max_workers:
                t = threading.Thread(target=self._work, name=f"{self.name}_{len(self._threads)}", daemon=True)
                self._threads.append(t)
                t.start()
            # else: every worker is busy and at the limit; the next one to finish takes it
        return fut

    def _work(self) -> None:
        while True:
            with self._cv:
                while not self._queue and not self._shutdown:
                    self._idle += 1
                    self._cv.wait()  # whoever notified took this worker off the idle count
                if not self._queue:
                    return
                fut, fn, args, kwargs = self._queue.popleft()
            try:
                res = fn(*args, **kwargs)
            except BaseException as e:  # noqa: BLE001 - delivered to the caller via the future
                fut._finish(exc=e)
            else:
                fut._finish(res)

    def map(self, fn, items) -> list:
        """Results in input order; the first failure (in input order) is raised."""
        return [f.result() for f in [self.submit(fn, x) for x in items]]

    def shutdown(self, wait: bool = True) -> None:
        with self._cv:
            self._shutdown = True
            self._cv.notify_all()
        if wait:
            me = threading.current_thread()
            for t in list(self._threads):
                if t is not me:
                    t.join()

    def __enter__(self) -> "Pool":
        return self

    def __exit__(self, *exc) -> None:
        self.shutdown(wait=True)


def as_completed(futures):
    """Yield the futures as they finish."""
    futures = list(futures)
    done: deque = deque()
    cv = threading.Condition()

    def cb(f):
        with cv:
            done.append(f)
            cv.notify()

    for f in futures:
        f.add_done_callback(cb)
    for _ in range(len(futures)):
        with cv:
            while not done:
                cv.wait()
            f = done.popleft()
        yield f
