"""The bundled kubectl's stream commands over the control plane's WebSocket channel endpoints:

* ``port-forward TARGET [LOCAL:]REMOTE ...`` -- TARGET is ``pod/NAME`` (or ``NAME``),
  ``deployment/NAME`` or ``service/NAME`` (a running pod the selector matches; a Service's port is
  mapped to its targetPort, as kubectl does). Every accepted local connection gets its own
  WebSocket (``v4.channel.k8s.io``, data channel 0, error channel 1).
* ``attach POD`` -- the pod's output from now on until it stops (output only).

What kubectl prints ("Forwarding from 127.0.0.1:8080 -> 80", "Handling connection for 8080") is
kept, so scripts that wait for that line work unchanged.
"""
from __future__ import annotations

import json
import socket
import sys
import threading
import time

from ..controlplane.wsclient import WSClient, WSClosed
from ..kube import kind_key, object_path


def _labels_match(sel: dict, labels: dict) -> bool:
    return all(labels.get(k) == v for k, v in (sel or {}).items())


def resolve_pod(k, target: str, ns: str, ports: list[int]) -> tuple[str, list[int]]:
    """TARGET -> (running pod name, remote ports after Service port -> targetPort mapping)."""
    what, name = target.split("/", 1) if "/" in target else ("pod", target)
    kind = kind_key(what)
    if kind == "pod":
        return name, ports
    obj = k.get(k.k8s(object_path(kind, name, ns)))
    if kind == "service":
        sel = obj["spec"].get("selector") or {}
        mapped = []
        for p in ports:
            sp = next((x for x in obj["spec"].get("ports", []) if x.get("port") == p), None)
            if sp is None:
                raise SystemExit(f"error: Service {name} does not have a service port {p}")
            tp = sp.get("targetPort", p)
            mapped.append(int(tp) if str(tp).isdigit() else p)
        ports = mapped
    elif kind in ("deployment", "daemonset", "job"):
        sel = (obj["spec"].get("selector") or {}).get("matchLabels") or {}
    else:
        raise SystemExit(f"error: cannot port-forward to {what}")
    pods = k.get(k.k8s(f"/api/v1/namespaces/{ns}/pods"))["items"]
    for p in sorted(pods, key=lambda p: p["metadata"]["name"]):
        if p.get("status", {}).get("phase") == "Running" and _labels_match(sel, p["metadata"].get("labels", {})):
            return p["metadata"]["name"], ports
    raise SystemExit(f"error: no running pod for {target}")


def _pump_ws_to_sock(ws: WSClient, conn: socket.socket, port: int, last: list[float]) -> None:
    headers = 0
    try:
        while (msg := ws.recv()) is not None:
            last[0] = time.monotonic()
            if not msg:
                continue
            ch, data = msg[0], msg[1:]
            if headers < 2 and len(data) == 2:  # the two port frames that open the stream
                headers += 1
                continue
            if ch == 0:
                conn.sendall(data)
            elif ch == 1 and data:
                print(f"E port-forward {port}: {data.decode(errors='replace')}", file=sys.stderr, flush=True)
    except OSError:
        pass
    finally:
        try:
            conn.shutdown(socket.SHUT_WR)
        except OSError:
            pass


def _forward_one(k, pod: str, ns: str, remote: int, conn: socket.socket) -> None:
    try:
        ws = WSClient.connect(k.host, k.port, k.k8s(object_path("pod", pod, ns) + "/portforward"),
                              [("ports", str(remote))], k.token, ("v4.channel.k8s.io",))
    except (OSError, WSClosed) as e:
        print(f"E port-forward {remote}: {e}", file=sys.stderr, flush=True)
        conn.close()
        return
    last = [time.monotonic()]
    t = threading.Thread(target=_pump_ws_to_sock, args=(ws, conn, remote, last), daemon=True)
    t.start()
    try:
        while chunk := conn.recv(1 << 16):
            ws.send(b"\x00" + chunk)
    except OSError:
        pass
    # The local side is done sending. The channel protocol has no half-close, so keep relaying
    # the pod's answer while it still comes (0.5 s without data ends it), then close the stream.
    deadline = time.monotonic() + 30
    while t.is_alive() and time.monotonic() < deadline and time.monotonic() - last[0] < 0.5:
        t.join(0.1)
    ws.close()
    conn.close()


def port_forward(k, ns: str, target: str, specs: list[str], address: str = "127.0.0.1") -> int:
    if not specs:
        raise SystemExit("usage: kubectl port-forward TYPE/NAME [LOCAL_PORT:]REMOTE_PORT ...")
    pairs = []
    for sp in specs:
        local, _, remote = sp.rpartition(":")
        pairs.append((int(local) if local else (0 if ":" in sp else int(remote)), int(remote)))
    pod, remotes = resolve_pod(k, target, ns, [r for _l, r in pairs])
    listeners = []
    for (local, _r), remote in zip(pairs, remotes):
        s = socket.socket(socket.AF_INET6 if ":" in address else socket.AF_INET)
        s.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
        s.bind((address, local))
        s.listen(64)
        print(f"Forwarding from {address}:{s.getsockname()[1]} -> {remote}", flush=True)
        listeners.append((s, remote))

    def serve(s: socket.socket, remote: int):
        while True:
            try:
                conn, _ = s.accept()
            except OSError:
                return
            print(f"Handling connection for {s.getsockname()[1]}", flush=True)
            threading.Thread(target=_forward_one, args=(k, pod, ns, remote, conn), daemon=True).start()

    threads = [threading.Thread(target=serve, args=ls, daemon=True) for ls in listeners]
    for t in threads:
        t.start()
    try:
        for t in threads:
            t.join()
    except KeyboardInterrupt:
        pass
    return 0


def attach(k, ns: str, pod: str) -> int:
    """Stream the pod's output (channel 1) until its Status (channel 3)."""
    try:
        ws = WSClient.connect(k.host, k.port, k.k8s(object_path("pod", pod, ns) + "/attach"),
                              [("stdout", "true"), ("stderr", "true")], k.token,
                              ("v5.channel.k8s.io", "v4.channel.k8s.io"))
    except (OSError, WSClosed) as e:
        print(f"error: {e}", file=sys.stderr)
        return 1
    code = 0
    try:
        while (msg := ws.recv()) is not None:
            if msg[:1] == b"\x01":
                sys.stdout.buffer.write(msg[1:])
                sys.stdout.flush()
            elif msg[:1] == b"\x02":
                sys.stderr.buffer.write(msg[1:])
            elif msg[:1] == b"\x03":
                st = json.loads(msg[1:] or b"{}")
                code = 0 if st.get("status") == "Success" else 1
                if code:
                    print(f"error: {st.get('message', 'attach ended')}", file=sys.stderr)
                break
    except KeyboardInterrupt:
        pass
    ws.close()
    return code


def exec_tty(k, ns: str, pod: str, command: list[str], stdin: bool = True, inp=None, out=None) -> int:
    """``kubectl exec -it POD -- CMD``: a pseudo-terminal in the pod (k8s_api.h_pod_exec_ws with
    tty=true). This terminal goes raw while it runs, its size is sent first and on every SIGWINCH
    (channel 4), keystrokes go on channel 0, the pod's terminal output comes back on channel 1;
    the exit code is the command's."""
    q = [("command", c) for c in command] + [("stdout", "true"), ("tty", "true")]
    if stdin:
        q.append(("stdin", "true"))
    return _interactive(k, object_path("pod", pod, ns) + "/exec", q, stdin, True, inp, out)


def attach_interactive(k, ns: str, pod: str, stdin: bool, tty: bool, container: str | None = None,
                       inp=None, out=None, quiet: bool = False) -> int:
    """``kubectl attach -i [-t] POD`` (and ``kubectl run -it``): a session on the container's own
    stdin and output (k8s_api.h_pod_attach_ws with stdin/tty: the node agent's
    ``_run_attach_stream``); with ``-t`` this terminal goes raw like ``exec -it``. The exit code is
    the container's when it ends during the session."""
    q = [("stdout", "true"), ("stderr", "true")]
    q += [("stdin", "true")] if stdin else []
    q += [("tty", "true")] if tty else []
    q += [("container", container)] if container else []
    if tty and not quiet:
        print("If you don't see a command prompt, try pressing enter.", file=sys.stderr)
    return _interactive(k, object_path("pod", pod, ns) + "/attach", q, stdin, tty, inp, out)


def _interactive(k, path: str, q: list, stdin: bool, tty: bool, inp=None, out=None) -> int:
    import os
    import signal
    import threading

    inp = sys.stdin if inp is None else inp
    out = sys.stdout.buffer if out is None else out
    try:
        ws = WSClient.connect(k.host, k.port, k.k8s(path), q, k.token,
                              ("v5.channel.k8s.io", "v4.channel.k8s.io"), timeout=30)
    except (OSError, WSClosed) as e:
        print(f"error: {e}", file=sys.stderr)
        return 1
    lock = threading.Lock()

    def send(b: bytes) -> None:
        with lock:
            try:
                ws.send(b)
            except OSError:
                pass

    fd = inp.fileno() if hasattr(inp, "fileno") else None
    is_tty = tty and fd is not None and os.isatty(fd)

    def resize(*_):
        try:
            sz = os.get_terminal_size(fd)
            send(b"\x04" + json.dumps({"Width": sz.columns, "Height": sz.lines}).encode())
        except OSError:
            pass

    saved = None
    if is_tty:
        import termios
        import tty as _tty

        saved = termios.tcgetattr(fd)
        _tty.setraw(fd)
        resize()
        old_winch = signal.signal(signal.SIGWINCH, resize)

    def pump():
        while True:
            try:
                data = os.read(fd, 4096) if fd is not None else inp.read(4096)
            except OSError:
                data = b""
            if not data:
                send(b"\xff\x00")  # stdin closed (v5)
                return
            send(b"\x00" + (data if isinstance(data, bytes) else data.encode()))

    if stdin:
        threading.Thread(target=pump, name="exec-stdin", daemon=True).start()
    code = 1
    try:
        while (msg := ws.recv()) is not None:
            if msg[:1] in (b"\x01", b"\x02"):
                out.write(msg[1:])
                out.flush()
            elif msg[:1] == b"\x03":
                st = json.loads(msg[1:] or b"{}")
                code = 0 if st.get("status") == "Success" else 1
                for c in ((st.get("details") or {}).get("causes") or []):
                    if c.get("reason") == "ExitCode":
                        code = int(c.get("message") or 1)
                if st.get("status") != "Success" and st.get("reason") != "NonZeroExitCode":
                    print(f"error: {st.get('message', 'exec failed')}", file=sys.stderr)
                break
    except KeyboardInterrupt:
        pass
    finally:
        if saved is not None:
            import termios

            termios.tcsetattr(fd, termios.TCSADRAIN, saved)
            signal.signal(signal.SIGWINCH, old_winch)
        ws.close()
    return code
