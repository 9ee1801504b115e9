"""Cluster DNS (the ``dns`` container of the reference's Rancher Kubernetes stack,
docs/img/infrastructure-containers.png): authoritative A records under ``cluster.local``.

  <svc>.<ns>.svc.cluster.local   (also <svc>.<ns>.svc and <svc>.<ns>)   -> the Service's clusterIP
                                 (a headless Service, clusterIP None: its running pods' IPs)
  <host>.<svc>.<ns>.svc.cluster.local                                  -> the pod with that hostname
                                 and subdomain (a StatefulSet's <name>-<ordinal> under its Service)
  <a-b-c-d>.<ns>.pod.cluster.local                                     -> a.b.c.d
  <svc>.<ns>.svc.cluster.local of an ExternalName Service              -> a CNAME to its externalName
  any other name under cluster.local                                   -> NXDOMAIN
  names outside the cluster domain                                     -> REFUSED (not a recursor)

Served over UDP by the control plane on the master address (port 53, shifted by
utils.net.host_port when not root). Process pods share the host's resolver, so they discover
Services through the kubelet-style env vars; this answers tools and clients pointed at it
(``dig @<master> -p <port> frontend.default.svc.cluster.local``).
"""
from __future__ import annotations

import asyncio
import socket
import struct
from typing import Callable

DOMAIN = "cluster.local"
NOERROR, NXDOMAIN, REFUSED, FORMERR = 0, 3, 5, 1
QTYPE_A, QTYPE_CNAME, QTYPE_ANY, QCLASS_IN = 1, 5, 255, 1


class CName(str):
    """A resolver answer that is an alias (an ExternalName Service): the target's name."""


def parse_query(data: bytes) -> tuple[int, int, list[str], int, int, bytes]:
    """(id, flags, labels, qtype, qclass, question section) of a single-question query."""
    if len(data) < 12:
        raise ValueError("short DNS header")
    qid, flags, qd, _, _, _ = struct.unpack("!HHHHHH", data[:12])
    if qd != 1:
        raise ValueError("exactly one question expected")
    i, labels = 12, []
    while True:
        n = data[i]
        i += 1
        if n == 0:
            break
        if n & 0xC0:
            raise ValueError("compressed name in a question")
        labels.append(data[i:i + n].decode("ascii", "replace").lower())
        i += n
    qtype, qclass = struct.unpack("!HH", data[i:i + 4])
    return qid, flags, labels, qtype, qclass, data[12:i + 4]


def _name(n: str) -> bytes:
    return b"".join(bytes([len(p)]) + p.encode() for p in n.rstrip(".").split(".") if p) + b"\x00"


def build_reply(qid: int, flags: int, question: bytes, rcode: int, ips: list[str], ttl: int = 5,
                cname: str | None = None) -> bytes:
    answers = []
    if cname:
        target = _name(cname)
        answers.append(b"\xc0\x0c" + struct.pack("!HHIH", QTYPE_CNAME, QCLASS_IN, ttl, len(target)) + target)
    answers += [b"\xc0\x0c" + struct.pack("!HHIH", QTYPE_A, QCLASS_IN, ttl, 4) + socket.inet_aton(ip) for ip in ips]
    hdr = struct.pack("!HHHHHH", qid, 0x8000 | 0x0400 | (flags & 0x0100) | rcode, 1, len(answers), 0, 0)
    return hdr + question + b"".join(answers)


def _read_name(data: bytes, i: int) -> str:
    parts = []
    while data[i]:
        if data[i] & 0xC0:
            return ".".join(parts + [_read_name(data, ((data[i] & 0x3F) << 8) | data[i + 1])])
        parts.append(data[i + 1:i + 1 + data[i]].decode())
        i += data[i] + 1
    return ".".join(parts)


def query(name: str, qid: int = 0x1234) -> bytes:
    """A one-question A query (tests and ``tk8s`` tools)."""
    q = b"".join(bytes([len(p)]) + p.encode() for p in name.rstrip(".").split(".")) + b"\x00"
    return struct.pack("!HHHHHH", qid, 0x0100, 1, 0, 0, 0) + q + struct.pack("!HH", QTYPE_A, QCLASS_IN)


def parse_reply(data: bytes, cnames: list | None = None) -> tuple[int, list[str]]:
    """(rcode, A addresses) of a reply to ``query``; CNAME targets are appended to ``cnames``."""
    _, flags, _, an, _, _ = struct.unpack("!HHHHHH", data[:12])
    i = 12
    while data[i]:
        i += data[i] + 1
    i += 5
    ips = []
    for _ in range(an):
        i += 2  # name pointer
        rtype, _, _, rdlen = struct.unpack("!HHIH", data[i:i + 10])
        i += 10
        if rtype == QTYPE_A and rdlen == 4:
            ips.append(socket.inet_ntoa(data[i:i + 4]))
        elif rtype == QTYPE_CNAME and cnames is not None:
            cnames.append(_read_name(data, i))
        i += rdlen
    return flags & 0xF, ips


class DnsProtocol(asyncio.DatagramProtocol):
    def __init__(self, resolve: Callable[[str], list[str] | None | bool]):
        self.resolve = resolve   # name -> [ips] | None (NXDOMAIN) | False (REFUSED)
        self.transport = None

    def connection_made(self, transport) -> None:
        self.transport = transport

    def datagram_received(self, data: bytes, addr) -> None:
        try:
            qid, flags, labels, qtype, qclass, question = parse_query(data)
        except (ValueError, IndexError, struct.error):
            return
        ips = self.resolve(".".join(labels))
        if ips is False:
            reply = build_reply(qid, flags, question, REFUSED, [])
        elif ips is None:
            reply = build_reply(qid, flags, question, NXDOMAIN, [])
        elif isinstance(ips, CName):  # an alias answers every type with the CNAME
            reply = build_reply(qid, flags, question, NOERROR, [], cname=str(ips))
        elif qclass == QCLASS_IN and qtype in (QTYPE_A, QTYPE_ANY):
            reply = build_reply(qid, flags, question, NOERROR, ips)
        else:
            reply = build_reply(qid, flags, question, NOERROR, [])  # name exists, no record of that type
        self.transport.sendto(reply, addr)
