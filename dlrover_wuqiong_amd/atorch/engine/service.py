"""Acceleration-engine service (rank 0) and its client (every rank).

The engine serves the executor over the framework's generic gRPC transport
(``common/rpc.py``: one ``get`` and one ``report`` method carrying JSON);
messages are ``{"op": "get_task", "process_id": p}`` and
``{"op": "report", "task_id", "process_id", "task_type", "ok", "result"}``.

Parity: reference ``atorch/atorch/auto/engine/acceleration_engine.py``
(``AccelerationEngine``: create executor, start_service, tear_down),
``auto/engine/servicer.py`` (``AutoAccelerationService``) and
``auto/engine/client.py`` / ``auto/engine_client.py`` (``EngineClient``).
"""

import os
import time
from typing import Optional

from ...common.log import logger
from ...common.rpc import RpcClient, RpcServer
from .executor import Executor
from .task import Task, decode, dumps, encode, loads


class AccelerationEngine:
    def __init__(self, device_context, included_opts=None, excluded_opts=None, time_limit=None,
                 load_strategy=None, verbose: bool = False):
        self.executor = Executor(device_context, included_opts=included_opts, excluded_opts=excluded_opts,
                                 time_limit=time_limit, load_strategy=load_strategy, verbose=verbose)
        self.port: Optional[int] = None
        self.server: Optional[RpcServer] = None

    def _get(self, req: bytes) -> bytes:
        msg = loads(req)
        if msg.get("op") != "get_task":
            raise ValueError(f"unknown engine request {msg.get('op')}")
        return dumps(self.executor.get_task(int(msg["process_id"])).wire())

    def _report(self, req: bytes) -> bytes:
        msg = loads(req)
        self.executor.report_task_result(int(msg["task_id"]), int(msg["process_id"]), bool(msg["ok"]),
                                         decode(msg.get("result")))
        return b"{}"

    def start_service(self, port: int = 0) -> int:
        self.server = RpcServer(port, report=self._report, get=self._get,
                                max_workers=max(8, self.executor.total_process + 2))
        self.port = self.server.port
        self.server.start()
        logger.info(f"acceleration engine serving on port {self.port}")
        return self.port

    def tear_down(self, force: bool = False, timeout: float = 120.0):
        deadline = time.time() + timeout
        while not force and not self.executor.can_be_terminated and time.time() < deadline:
            time.sleep(0.05)
        if not self.executor.can_be_terminated:
            logger.warning("acceleration engine stopped before every process got its final task")
        if self.server is not None:
            self.server.stop(0.5)
            self.server = None

    def service_port(self) -> Optional[int]:
        return self.port


class EngineClient:
    def __init__(self, addr: Optional[str] = None, port: Optional[int] = None, process_id: Optional[int] = None,
                 timeout: float = 60.0):
        addr = addr or os.getenv("MASTER_ADDR", "127.0.0.1")
        self.process_id = int(os.getenv("RANK", "0")) if process_id is None else int(process_id)
        self.rpc = RpcClient(f"{addr}:{port}", timeout=timeout)

    def get_task(self) -> Task:
        w = loads(self.rpc.get(dumps({"op": "get_task", "process_id": self.process_id})))
        return Task(w["task_type"], decode(w["info"]), task_id=w["task_id"], process_mode=w["process_mode"],
                    time_limit=w["time_limit"])

    def report_task_result(self, task: Task, ok: bool, result=None):
        self.rpc.report(dumps({"op": "report", "task_id": task.task_id, "process_id": self.process_id,
                               "task_type": task.task_type, "ok": bool(ok), "result": encode(result)}))

    def close(self):
        self.rpc.close()
