"""Named syncs / barriers through the job master.

Parity: reference ``dlrover/python/elastic_agent/sychronization/sync_client.py:19-74``.
"""

import time
from typing import Optional

from ..common.log import logger
from .master_client import MasterClient


class SyncClient:
    def __init__(self, master_client: Optional[MasterClient] = None):
        self._mc = master_client or MasterClient.singleton_instance()

    def join_sync(self, sync_name: str) -> bool:
        """Join a named sync; True once the master accepted the join."""
        ok = self._mc.join_sync(sync_name)
        logger.info(f"joined sync {sync_name}: {ok}")
        return ok

    def sync_finished(self, sync_name: str) -> bool:
        return self._mc.sync_finished(sync_name)

    def barrier(self, barrier_name: str, timeout: float = 3600.0, poll: float = 1.0) -> bool:
        """Block until some process notifies the barrier (or timeout)."""
        deadline = time.time() + timeout
        while time.time() < deadline:
            if self._mc.barrier(barrier_name):
                return True
            time.sleep(poll)
        return False

    def notify_barrier(self, barrier_name: str) -> bool:
        return self._mc.barrier(barrier_name, notify=True)

    def wait_sync(self, sync_name: str, timeout: float = 3600.0, poll: float = 1.0) -> bool:
        """Join then wait until every running node has joined."""
        self.join_sync(sync_name)
        deadline = time.time() + timeout
        while time.time() < deadline:
            if self.sync_finished(sync_name):
                return True
            time.sleep(poll)
        return False
