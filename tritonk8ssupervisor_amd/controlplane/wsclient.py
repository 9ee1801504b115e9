"""A small blocking WebSocket client (RFC 6455) for the bundled kubectl's stream commands --
``port-forward`` and ``attach`` -- against the control plane's channel protocol endpoints
(k8s_api.h_pod_portforward_ws / h_pod_attach_ws). Client frames are masked, as the RFC requires;
messages are sent unfragmented; pings are answered."""
from __future__ import annotations

import base64
import os
import socket
from urllib.parse import urlencode


class WSClosed(Exception):
    pass


class WSClient:
    def __init__(self, sock: socket.socket, protocol: str):
        self.sock, self.protocol = sock, protocol
        self._buf = b""

    @classmethod
    def connect(cls, host: str, port: int, path: str, query: list[tuple[str, str]] | None = None,
                token: str | None = None, protocols: tuple[str, ...] = (), timeout: float = 10.0) -> "WSClient":
        sock = socket.create_connection((host, port), timeout=timeout)
        key = base64.b64encode(os.urandom(16)).decode()
        target = path + ("?" + urlencode(query) if query else "")
        lines = [f"GET {target} HTTP/1.1", f"Host: {host}:{port}", "Upgrade: websocket", "Connection: Upgrade",
                 f"Sec-WebSocket-Key: {key}", "Sec-WebSocket-Version: 13"]
        if protocols:
            lines.append("Sec-WebSocket-Protocol: " + ", ".join(protocols))
        if token:
            lines.append(f"Authorization: Bearer {token}")
        sock.sendall(("\r\n".join(lines) + "\r\n\r\n").encode())
        head = b""
        while b"\r\n\r\n" not in head:
            chunk = sock.recv(4096)
            if not chunk:
                raise WSClosed("connection closed during the upgrade")
            head += chunk
        head, rest = head.split(b"\r\n\r\n", 1)
        status_line, *hdrs = head.decode(errors="replace").split("\r\n")
        if " 101 " not in status_line + " ":
            body = rest
            try:
                sock.settimeout(2)
                while chunk := sock.recv(65536):
                    body += chunk
            except OSError:
                pass
            sock.close()
            raise WSClosed(f"{status_line}: {body.decode(errors='replace')[:500]}")
        headers = {h.split(":", 1)[0].strip().lower(): h.split(":", 1)[1].strip() for h in hdrs if ":" in h}
        sock.settimeout(None)
        ws = cls(sock, headers.get("sec-websocket-protocol", ""))
        ws._buf = rest
        return ws

    def _read(self, n: int) -> bytes:
        while len(self._buf) < n:
            chunk = self.sock.recv(max(65536, n - len(self._buf)))
            if not chunk:
                raise WSClosed("connection closed")
            self._buf += chunk
        out, self._buf = self._buf[:n], self._buf[n:]
        return out

    def send(self, data: bytes, opcode: int = 0x2) -> None:
        n = len(data)
        head = bytes([0x80 | opcode])
        if n < 126:
            head += bytes([0x80 | n])
        elif n < 1 << 16:
            head += bytes([0x80 | 126]) + n.to_bytes(2, "big")
        else:
            head += bytes([0x80 | 127]) + n.to_bytes(8, "big")
        mask = os.urandom(4)
        if n:
            m = (mask * (n // 4 + 1))[:n]
            data = (int.from_bytes(data, "little") ^ int.from_bytes(m, "little")).to_bytes(n, "little")
        self.sock.sendall(head + mask + data)

    def recv(self) -> bytes | None:
        """The next message; None when the server closed the stream."""
        buf = b""
        while True:
            try:
                h = self._read(2)
            except (WSClosed, OSError):
                return None
            fin, opcode, n = h[0] & 0x80, h[0] & 0x0F, h[1] & 0x7F
            if n == 126:
                n = int.from_bytes(self._read(2), "big")
            elif n == 127:
                n = int.from_bytes(self._read(8), "big")
            data = self._read(n)
            if opcode == 0x8:
                try:
                    self.send(data[:2], 0x8)
                except OSError:
                    pass
                return None
            if opcode == 0x9:
                self.send(data, 0xA)
                continue
            if opcode == 0xA:
                continue
            buf += data
            if fin:
                return buf

    def close(self) -> None:
        try:
            self.send((1000).to_bytes(2, "big"), 0x8)
        except OSError:
            pass
        try:
            self.sock.close()
        except OSError:
            pass
