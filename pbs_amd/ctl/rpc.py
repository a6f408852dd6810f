"""Length-prefixed JSON-RPC over a Unix socket (the privcmd ioctl ->
domctl/sysctl path of the reference, X:tools/libxc/xc_linux_osdep.c:116).

Frame: 4-byte big-endian length + UTF-8 JSON.  Request {"method", "params"},
reply {"ok": true, "result": ...} or {"ok": false, "error": str, "code": int}.
"""
from __future__ import annotations

import json
import os
import socket
import socketserver
import struct
import threading
from typing import Any, Callable, Dict

DEFAULT_SOCKET = os.environ.get("GPBS_SOCKET", "/tmp/gpbsd.sock")


class RpcError(RuntimeError):
    def __init__(self, msg: str, code: int = -1):
        super().__init__(msg)
        self.code = code


def _send(sock, obj):
    data = json.dumps(obj).encode()
    sock.sendall(struct.pack(">I", len(data)) + data)


def _recv_exact(sock, n):
    buf = b""
    while len(buf) < n:
        chunk = sock.recv(n - len(buf))
        if not chunk:
            raise ConnectionError("peer closed")
        buf += chunk
    return buf


def _recv(sock):
    (n,) = struct.unpack(">I", _recv_exact(sock, 4))
    return json.loads(_recv_exact(sock, n).decode())


class Client:
    def __init__(self, path: str = DEFAULT_SOCKET, timeout: float = 30.0):
        self.path = path
        self.sock = socket.socket(socket.AF_UNIX, socket.SOCK_STREAM)
        self.sock.settimeout(timeout)
        self.sock.connect(path)
        self.lock = threading.Lock()

    def call(self, method: str, **params) -> Any:
        with self.lock:
            _send(self.sock, {"method": method, "params": params})
            rep = _recv(self.sock)
        if not rep.get("ok"):
            raise RpcError(rep.get("error", "rpc error"), rep.get("code", -1))
        return rep.get("result")

    def close(self):
        try:
            self.sock.close()
        except OSError:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()


class Server:
    """Threaded RPC server dispatching to ``handlers[method](**params)``."""

    def __init__(self, path: str, handlers: Dict[str, Callable[..., Any]]):
        self.path = path
        self.handlers = handlers
        if os.path.exists(path):
            os.unlink(path)
        outer = self

        class H(socketserver.BaseRequestHandler):
            def handle(self):
                while True:
                    try:
                        req = _recv(self.request)
                    except (ConnectionError, OSError, struct.error):
                        return
                    m = req.get("method")
                    fn = outer.handlers.get(m)
                    try:
                        if fn is None:
                            raise RpcError(f"unknown method '{m}'", -38)
                        res = fn(**(req.get("params") or {}))
                        _send(self.request, {"ok": True, "result": res})
                    except Exception as e:  # report to the caller, keep serving
                        _send(self.request, {"ok": False, "error": str(e), "code": getattr(e, "code", -1)})

        class S(socketserver.ThreadingMixIn, socketserver.UnixStreamServer):
            daemon_threads = True

        self.srv = S(path, H)
        os.chmod(path, 0o600)
        self.thread = threading.Thread(target=self.srv.serve_forever, daemon=True)

    def start(self):
        self.thread.start()
        return self

    def stop(self):
        self.srv.shutdown()
        self.srv.server_close()
        if os.path.exists(self.path):
            os.unlink(self.path)
