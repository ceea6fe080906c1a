"""A c10d ``Store`` backed by the job master's KV service.

Lets ``torch.distributed`` rendezvous (the TCPStore-less path) go through the
master, exactly like reference
``dlrover/python/elastic_agent/torch/master_kv_store.py:23-150``.
"""

import time
from datetime import timedelta
from typing import List, Optional

import torch.distributed as dist

from .master_client import MasterClient


class MasterKVStore(dist.Store):
    def __init__(self, client: MasterClient, prefix: str = "", timeout: timedelta = timedelta(seconds=300)):
        super().__init__()
        self.client = client
        self.prefix = prefix
        self.timeout = timeout

    def _k(self, key: str) -> str:
        return self.prefix + key

    def set(self, key: str, value):
        if isinstance(value, str):
            value = value.encode()
        self.client.kv_store_set(self._k(key), bytes(value))

    def get(self, key: str) -> bytes:
        deadline = time.time() + self.timeout.total_seconds()
        while True:
            v = self.client.kv_store_get(self._k(key))
            if v:
                return v
            if time.time() > deadline:
                raise LookupError(f"key {key} not found in master KV store within {self.timeout}")
            time.sleep(0.05)

    def add(self, key: str, amount: int) -> int:
        return self.client.kv_store_add(self._k(key), amount)

    def compare_set(self, key: str, expected, desired) -> bytes:
        cur = self.client.kv_store_get(self._k(key))
        exp = expected.encode() if isinstance(expected, str) else expected
        des = desired.encode() if isinstance(desired, str) else desired
        if cur == exp or (not cur and not exp):
            self.client.kv_store_set(self._k(key), des)
            return des
        return cur

    def wait(self, keys: List[str], timeout: Optional[timedelta] = None):
        t = (timeout or self.timeout).total_seconds()
        deadline = time.time() + t
        for k in keys:
            while not self.client.kv_store_get(self._k(k)):
                if time.time() > deadline:
                    raise LookupError(f"wait for {k} timed out")
                time.sleep(0.05)

    def check(self, keys: List[str]) -> bool:
        return all(bool(self.client.kv_store_get(self._k(k))) for k in keys)

    def delete_key(self, key: str) -> bool:
        self.client.kv_store_set(self._k(key), b"")
        return True

    def num_keys(self) -> int:
        return 0

    def set_timeout(self, timeout: timedelta):
        self.timeout = timeout
