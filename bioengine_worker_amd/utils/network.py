"""Network helpers (reference: bioengine/utils/network.py:8-118).

``get_internal_ip`` prefers RFC1918 interface addresses (enumerated with SIOCGIFADDR);
``acquire_free_port`` scans upward from a start port and can keep the probe socket open so that a
concurrent scan in another process cannot take the same port.
"""
from __future__ import annotations

import ipaddress
import socket
import struct

try:
    import fcntl
except ImportError:  # pragma: no cover
    fcntl = None


def _interface_ips() -> list[str]:
    ips = []
    if fcntl is None:
        return ips
    try:
        names = [n for _, n in socket.if_nameindex()]
    except OSError:
        return ips
    s = socket.socket(socket.AF_INET, socket.SOCK_DGRAM)
    try:
        for name in names:
            try:
                req = struct.pack("256s", name[:15].encode())
                res = fcntl.ioctl(s.fileno(), 0x8915, req)  # SIOCGIFADDR
                ips.append(socket.inet_ntoa(res[20:24]))
            except OSError:
                continue
    finally:
        s.close()
    return ips


def get_internal_ip() -> str:
    ips = [ip for ip in _interface_ips() if not ip.startswith("127.")]
    private = [ip for ip in ips if ipaddress.ip_address(ip).is_private]
    if private:
        return private[0]
    if ips:
        return ips[0]
    try:
        return socket.gethostbyname(socket.gethostname())
    except OSError:
        return "127.0.0.1"


def acquire_free_port(port: int = 0, step: int = 1, ip: str = "127.0.0.1", keep_open: bool = False, max_tries: int = 2000):
    """Return a free port >= ``port`` (or an ephemeral one for 0).  With ``keep_open`` returns
    ``(port, socket)`` and the caller closes the socket right before binding the real server."""
    if port == 0:
        s = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
        s.bind((ip, 0))
        p = s.getsockname()[1]
        if keep_open:
            return p, s
        s.close()
        return p
    p = port
    for _ in range(max_tries):
        s = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
        try:
            s.bind((ip, p))
        except OSError:
            s.close()
            p += step
            continue
        if keep_open:
            return p, s
        s.close()
        return p
    raise RuntimeError(f"no free port found from {port}")
