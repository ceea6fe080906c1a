"""gRPC transport for the master service (no generated stubs needed).

One service ``dwamd.Master`` with two unary methods, ``report`` and ``get``,
both carrying a serialized :class:`comm.BaseRequest` envelope (JSON) - the
same two-verb design as the reference (``dlrover/proto/elastic_training.proto
:26-29``) but without protoc-generated code or pickled payloads.

Parity: reference ``dlrover/python/common/grpc.py`` (``build_channel`` :30,
``addr_connected`` :54, ``find_free_port*`` :71-105) and the 256 MB message
limit of ``constants.GRPC``.
"""

import socket
from concurrent import futures
from contextlib import closing
from typing import Callable, Optional

import grpc

from .constants import GRPC

SERVICE = "dwamd.Master"
_OPTS = [
    ("grpc.max_send_message_length", GRPC.MAX_SEND_MESSAGE_LENGTH),
    ("grpc.max_receive_message_length", GRPC.MAX_RECEIVE_MESSAGE_LENGTH),
    ("grpc.enable_retries", 1),
]


def _ident(b):
    return b


def build_channel(addr: str) -> Optional[grpc.Channel]:
    if not addr:
        return None
    return grpc.insecure_channel(addr, options=_OPTS)


def addr_connected(addr: str, timeout: float = 2.0) -> bool:
    if not addr or ":" not in addr:
        return False
    host, port = addr.rsplit(":", 1)
    try:
        with closing(socket.create_connection((host, int(port)), timeout=timeout)):
            return True
    except OSError:
        return False


def find_free_port(port: int = 0) -> int:
    with closing(socket.socket(socket.AF_INET, socket.SOCK_STREAM)) as s:
        s.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
        s.bind(("", port))
        return s.getsockname()[1]


def find_free_port_in_range(start: int, end: int) -> int:
    # scan from a random offset: concurrent jobs probing in the same order
    # would all pick the first free port (probe-then-bind race)
    import random

    n = end - start
    off = random.SystemRandom().randrange(n) if n > 0 else 0
    for i in range(n):
        p = start + (off + i) % n
        try:
            return find_free_port(p)
        except OSError:
            continue
    raise RuntimeError(f"no free port in [{start}, {end})")


def find_free_port_in_set(ports) -> int:
    for p in ports:
        try:
            return find_free_port(int(p))
        except OSError:
            continue
    raise RuntimeError(f"no free port in {ports}")


class RpcServer:
    """Serves ``report(bytes)->bytes`` and ``get(bytes)->bytes``."""

    def __init__(self, port: int, report: Callable[[bytes], bytes], get: Callable[[bytes], bytes],
                 max_workers: int = 64):
        self.server = grpc.server(futures.ThreadPoolExecutor(max_workers=max_workers), options=_OPTS)
        handlers = {
            "report": grpc.unary_unary_rpc_method_handler(lambda req, ctx: report(req), _ident, _ident),
            "get": grpc.unary_unary_rpc_method_handler(lambda req, ctx: get(req), _ident, _ident),
        }
        self.server.add_generic_rpc_handlers((grpc.method_handlers_generic_handler(SERVICE, handlers),))
        self.port = self.server.add_insecure_port(f"[::]:{port}")

    def start(self):
        self.server.start()

    def stop(self, grace: float = 0.5):
        self.server.stop(grace)


class RpcClient:
    def __init__(self, addr: str, timeout: float = 10.0):
        self.addr = addr
        self.timeout = timeout
        self.channel = build_channel(addr)
        self._report = self.channel.unary_unary(f"/{SERVICE}/report", request_serializer=_ident,
                                                response_deserializer=_ident)
        self._get = self.channel.unary_unary(f"/{SERVICE}/get", request_serializer=_ident,
                                             response_deserializer=_ident)

    def report(self, data: bytes, timeout: Optional[float] = None) -> bytes:
        return self._report(data, timeout=timeout or self.timeout)

    def get(self, data: bytes, timeout: Optional[float] = None) -> bytes:
        return self._get(data, timeout=timeout or self.timeout)

    def close(self):
        self.channel.close()
