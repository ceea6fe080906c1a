"""Cross-node in-memory replicas of flash-checkpoint shards.

If a node is replaced, its shm is gone; with ``replica_count > 0`` the shard
also lives in the memory of ``replica_count - 1`` peer nodes and the new node
pulls it back instead of reading storage.

Parity: reference ``dlrover/trainer/torch/flash_checkpoint/replica.py``
(``ShardCkptReplicaManager`` :73-242 all-gathers the shm byte buffer in a
gloo group of ``replica_count`` nodes; ``FullCkptReplicaManager`` :245-350
broadcasts from any node holding a copy).

Only the latest complete slot of the (double-buffered) shard is shipped.

Backup groups: node n belongs to group n // replica_count; inside a group the
ranks with the same local rank exchange shards.  Peer shards are kept in a
separate shm segment per peer (``replica_{peer_rank}``) so a local restart
does not need the network at all.
"""

import pickle
from typing import List, Optional

import numpy as np
import torch
import torch.distributed as dist

from ..common import env_utils
from ..common.log import logger
from ..common.serialize import restricted_loads
from ..common.multi_process import SharedMemory
from .shm_handler import SharedMemoryHandler


class CkptReplicaManager:
    def __init__(self, engine, replica_count: int):
        self.replica_count = replica_count
        self.engine = engine
        self.local_rank = env_utils.get_local_rank()
        self.local_world = max(1, env_utils.get_local_world_size())
        self.node_rank = env_utils.get_node_rank()
        self.rank = dist.get_rank() if dist.is_available() and dist.is_initialized() else 0
        self.world = dist.get_world_size() if dist.is_available() and dist.is_initialized() else 1
        self.node_num = max(1, self.world // self.local_world)
        self._group = None
        self.backup_ranks: List[int] = []
        if replica_count > 1 and dist.is_available() and dist.is_initialized() and self.node_num > 1:
            self._build_groups()

    @staticmethod
    def create(engine, replica_count: int) -> "CkptReplicaManager":
        return CkptReplicaManager(engine, replica_count)

    def _build_groups(self):
        rc = self.replica_count
        n_groups = (self.node_num + rc - 1) // rc
        for g in range(n_groups):
            nodes = [n for n in range(g * rc, min(self.node_num, (g + 1) * rc))]
            for lr in range(self.local_world):
                ranks = [n * self.local_world + lr for n in nodes]
                pg = dist.new_group(ranks=ranks, backend="gloo")
                if self.rank in ranks:
                    self._group = pg
                    self.backup_ranks = ranks

    def has_replica(self) -> bool:
        return self._group is not None and len(self.backup_ranks) > 1

    # -------------------------------------------------------------- backup
    def backup(self, handler: SharedMemoryHandler):
        """All-gather every group member's shm bytes + metadata (gloo)."""
        if not self.has_replica():
            return
        self.engine.wait_for_memory_save()
        slot = handler.latest_slot() if handler.shared_memory is not None else -1
        if slot >= 0:
            view, meta = handler.export_slot(slot)
            payload = np.frombuffer(view, dtype=np.uint8)
        else:
            payload, meta = np.zeros(0, dtype=np.uint8), None
        size = torch.tensor([payload.size], dtype=torch.int64)
        sizes = [torch.zeros(1, dtype=torch.int64) for _ in self.backup_ranks]
        dist.all_gather(sizes, size, group=self._group)
        maxn = int(max(int(s) for s in sizes))
        buf = torch.zeros(max(maxn, 1), dtype=torch.uint8)
        buf[: payload.size] = torch.from_numpy(payload)
        outs = [torch.empty(max(maxn, 1), dtype=torch.uint8) for _ in self.backup_ranks]
        dist.all_gather(outs, buf, group=self._group)
        metas: List[Optional[dict]] = [None] * len(self.backup_ranks)
        dist.all_gather_object(metas, meta, group=self._group)
        for r, t, m, n in zip(self.backup_ranks, outs, metas, sizes):
            if r == self.rank or m is None:
                continue
            n = int(n)
            mb = pickle.dumps(m)
            # [4 KiB header: payload bytes, meta bytes][payload][meta]
            seg = SharedMemory(f"replica_{r}", create=True, size=4096 + n + len(mb))
            hdr = np.frombuffer(seg.buf, dtype=np.int64, count=2)
            seg.buf[4096: 4096 + n] = t[:n].numpy().tobytes()
            seg.buf[4096 + n: 4096 + n + len(mb)] = mb
            hdr[0] = n
            hdr[1] = len(mb)
            del hdr
            seg.close()

    # -------------------------------------------------------------- gather
    def gather(self, handler: SharedMemoryHandler):
        """Restore this rank's shm from a peer if it has none."""
        if not self.has_replica():
            return
        have = 1 if handler.complete_step() > 0 else 0
        flags = [torch.zeros(1, dtype=torch.int64) for _ in self.backup_ranks]
        dist.all_gather(flags, torch.tensor([have], dtype=torch.int64), group=self._group)
        if all(int(f) == 1 for f in flags):
            return
        # each member that holds a copy of a missing member's shard sends it
        for idx, (r, f) in enumerate(zip(self.backup_ranks, flags)):
            if int(f) == 1:
                continue
            # pick the first peer that has its own shard (i.e. is alive)
            donors = [self.backup_ranks[i] for i, ff in enumerate(flags) if int(ff) == 1]
            if not donors:
                continue
            donor = donors[0]
            obj = [None]
            if self.rank == donor:
                try:
                    seg = SharedMemory(f"replica_{r}")
                    hdr = np.frombuffer(seg.buf, dtype=np.int64, count=2)
                    n, mlen = int(hdr[0]), int(hdr[1])
                    del hdr
                    data = bytes(seg.buf[4096: 4096 + n])
                    meta = restricted_loads(bytes(seg.buf[4096 + n: 4096 + n + mlen])) if mlen else None
                    seg.close()
                    obj = [(data, meta)]
                except FileNotFoundError:
                    obj = [None]
            dist.broadcast_object_list(obj, src=donor, group=self._group)
            if self.rank == r and obj[0] is not None and obj[0][1]:
                data, meta = obj[0]
                handler.import_slot(data, meta)
                logger.info(f"rank {r} restored its checkpoint shard ({len(data)} B) from peer {donor}")
