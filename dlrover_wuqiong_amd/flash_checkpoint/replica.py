"""Cross-node in-memory replicas of flash-checkpoint shards.

If a node is replaced its shm is gone; with ``replica_count > 1`` every
shard also lives in the memory of the other ``replica_count - 1`` nodes of
its backup group, and the replacement node pulls it back instead of reading
storage.

Backup groups: node n belongs to group n // replica_count; inside a group
the ranks with the same local rank exchange shards (gloo, host memory).

Design (vs the reference's all_gather of whole padded payloads + pickled
metadata inside the save call):
  * off the training path: ``backup()`` only enqueues a ticket; a background
    thread waits until that step is complete in this rank's shm and ships
    it, so a save never waits for the network;
  * latest-only: a ticket every member of the group already holds a newer
    ticket for is dropped (one 8-byte all-reduce decides it collectively),
    so a slow link ships the newest checkpoint instead of a growing backlog;
  * torn-read free: the sender holds the shm slot's lock for the whole
    transfer (the save path writes the other slot meanwhile) and sends the
    slot's step again after the last chunk; the receiver marks the replica
    complete only if it matches;
  * raw chunked transfers: the payload moves in ``chunk``-byte pieces
    straight from this rank's shm slot into a persistent per-peer replica
    segment (``replica_{rank}``, re-created only when the size changes) --
    ``torch.frombuffer`` views on both sides, no pickling, no full-size
    staging tensor; a ring shift (round k: send to member i+k, receive from
    i-k with isend/irecv) keeps every link busy without deadlock;
  * crash-consistent: a replica's header step is zeroed before new bytes
    land and set after the confirmation, so a half-received copy is never used;
  * ``gather()`` (restore path) streams a missing member's shard from the
    first live peer holding it directly into the member's own shm slot.

Metadata (the layout tree + checkpoint config) is a small pickle read back
with the allow-listed unpickler.

Parity: reference ``dlrover/trainer/torch/flash_checkpoint/replica.py``
(``ShardCkptReplicaManager`` :73-242, ``FullCkptReplicaManager`` :245-350).
"""

import pickle
import queue
import threading
import time
from typing import List, Optional

import numpy as np
import torch
import torch.distributed as dist

from ..common import env_utils
from ..common.log import logger
from ..common.multi_process import SharedMemory
from ..common.serialize import restricted_loads
from .shm_handler import DLROVER_CKPT_CONFIG_KEY, SharedMemoryHandler

_HDR = 4096  # replica segment: [int64 step, payload bytes, meta bytes][...][payload][meta]
_CHUNK = 64 << 20


def _u8(buf, lo: int, hi: int) -> torch.Tensor:
    return torch.frombuffer(buf, dtype=torch.uint8, count=hi - lo, offset=lo) if hi > lo else torch.empty(
        0, dtype=torch.uint8)


class CkptReplicaManager:
    def __init__(self, engine, replica_count: int, chunk_bytes: int = _CHUNK):
        self.replica_count = replica_count
        self.engine = engine
        self.chunk = int(chunk_bytes)
        self.local_rank = env_utils.get_local_rank()
        self.local_world = max(1, env_utils.get_local_world_size())
        self.rank = dist.get_rank() if dist.is_available() and dist.is_initialized() else 0
        self.world = dist.get_world_size() if dist.is_available() and dist.is_initialized() else 1
        self.node_num = max(1, self.world // self.local_world)
        self._group = None
        self.backup_ranks: List[int] = []
        self._q: "queue.Queue" = queue.Queue()
        self._thread: Optional[threading.Thread] = None
        self._lock = threading.Lock()  # one user of the gloo group at a time
        self.last_backup = (0, 0.0)    # (step, seconds) of the last shipped backup
        self.coalesced = 0             # tickets skipped because every member held a newer one
        self.pin_timeout = 60.0        # max wait for a queued step to land in shm
        if replica_count > 1 and dist.is_available() and dist.is_initialized() and self.node_num > 1:
            self._build_groups()

    @staticmethod
    def create(engine, replica_count: int) -> "CkptReplicaManager":
        return CkptReplicaManager(engine, replica_count)

    def _build_groups(self):
        rc = self.replica_count
        n_groups = (self.node_num + rc - 1) // rc
        for g in range(n_groups):
            nodes = list(range(g * rc, min(self.node_num, (g + 1) * rc)))
            for lr in range(self.local_world):
                ranks = [n * self.local_world + lr for n in nodes]
                pg = dist.new_group(ranks=ranks, backend="gloo")  # every rank creates every group
                if self.rank in ranks:
                    self._group = pg
                    self.backup_ranks = ranks

    def has_replica(self) -> bool:
        return self._group is not None and len(self.backup_ranks) > 1

    @property
    def _me(self) -> int:
        return self.backup_ranks.index(self.rank)

    # -------------------------------------------------------------- backup
    def backup(self, handler: SharedMemoryHandler, step: Optional[int] = None):
        """Queue a ticket to ship this rank's checkpoint of ``step``
        (non-blocking).  Every member of the group calls this for the same
        saves, so every member's thread sees the same ticket sequence."""
        if not self.has_replica():
            return
        if self._thread is None:
            self._thread = threading.Thread(target=self._loop, args=(handler,), daemon=True,
                                            name="dwamd-ckpt-replica")
            self._thread.start()
        self._q.put(step if step is not None else getattr(self.engine, "_cached_step", 0))

    def wait(self, timeout: float = 600.0):
        """Block until every queued ticket has been handled."""
        if self._thread is None:
            return
        deadline = time.time() + timeout
        while self._q.unfinished_tasks and time.time() < deadline:
            time.sleep(0.01)

    def _loop(self, handler: SharedMemoryHandler):
        seq = 0
        while True:
            step = self._q.get()
            try:
                if step is None:
                    return
                seq += 1
                # latest-only coalescing, decided collectively: every member
                # processes ticket ``seq`` in the same order and votes the
                # newest ticket it already holds; if EVERY member already
                # holds a newer one, this ticket costs one 8-byte all-reduce
                # instead of shipping a payload that is about to be stale
                newest = seq + sum(1 for x in list(self._q.queue) if x is not None)
                t = torch.tensor([newest], dtype=torch.int64)
                dist.all_reduce(t, op=dist.ReduceOp.MIN, group=self._group)
                if int(t) > seq:
                    self.coalesced += 1
                    continue
                with self._lock:
                    t0 = time.perf_counter()
                    shipped = self._exchange(handler, step)
                    if shipped:
                        self.last_backup = (step, time.perf_counter() - t0)
            except Exception as e:  # pragma: no cover - logged, training continues
                logger.warning(f"checkpoint replica of step {step} failed: {e}")
            finally:
                self._q.task_done()

    def _pin_slot(self, handler: SharedMemoryHandler, step: int, timeout: float):
        """Wait until ``step`` is complete in shm, then hold that slot's lock
        (the save path never writes a locked slot) and return the slot; -1 if
        the step was superseded / overwritten first or never completed."""
        deadline = time.time() + timeout
        while time.time() < deadline:
            slot = handler.slot_of(step)
            if slot >= 0:
                lock = self.engine._shm_locks[slot]
                if not lock.acquire(blocking=True, timeout=max(0.0, deadline - time.time())):
                    return -1
                if handler.slot_step(slot) == step:
                    return slot
                lock.release()  # rewritten between the check and the lock
                continue
            if handler.complete_step() > step:
                return -1  # a newer checkpoint landed: this one is gone or going
            time.sleep(0.002)
        return -1

    def _exchange(self, handler: SharedMemoryHandler, step: int) -> bool:
        """One ring exchange of the group.  The sender holds its slot's lock
        for the whole transfer and confirms the step after the last chunk;
        the receiver stamps its replica complete only with that confirmation,
        so a torn copy is never served."""
        g = len(self.backup_ranks)
        slot = self._pin_slot(handler, step, float(self.pin_timeout))
        try:
            if slot >= 0:
                view, meta = handler.export_slot(slot)
                payload = memoryview(view)
                mb = pickle.dumps(meta)
            else:
                payload, mb = memoryview(b""), b""
            mine = torch.tensor([step if slot >= 0 else 0, len(payload), len(mb)], dtype=torch.int64)
            alls = [torch.zeros(3, dtype=torch.int64) for _ in range(g)]
            dist.all_gather(alls, mine, group=self._group)
            me = self._me
            for k in range(1, g):
                dst, src = (me + k) % g, (me - k) % g
                s_step, s_n, s_m = (int(x) for x in alls[src])
                seg = self._replica_segment(self.backup_ranks[src], s_n, s_m) if s_step > 0 else None
                hdr = np.frombuffer(seg.buf, dtype=np.int64, count=3) if seg is not None else None
                if hdr is not None:
                    hdr[0] = 0  # invalid until the last byte landed and the sender confirmed
                send_n = len(payload) if int(alls[me][0]) > 0 else 0
                reqs = []
                # metadata first, then the payload in chunks (isend/irecv
                # pairs: every member sends and receives in the same round)
                if send_n:
                    reqs.append(dist.isend(torch.frombuffer(bytearray(mb), dtype=torch.uint8),
                                           self.backup_ranks[dst], group=self._group))
                if seg is not None:
                    reqs.append(dist.irecv(_u8(seg.buf, _HDR + s_n, _HDR + s_n + s_m), self.backup_ranks[src],
                                           group=self._group))
                for r in reqs:
                    r.wait()
                n_chunks = max((send_n + self.chunk - 1) // self.chunk,
                               (s_n + self.chunk - 1) // self.chunk if seg else 0)
                for c in range(n_chunks):
                    reqs = []
                    lo = c * self.chunk
                    if lo < send_n:
                        hi = min(send_n, lo + self.chunk)
                        reqs.append(dist.isend(_u8(payload, lo, hi), self.backup_ranks[dst], group=self._group))
                    if seg is not None and lo < s_n:
                        hi = min(s_n, lo + self.chunk)
                        reqs.append(dist.irecv(_u8(seg.buf, _HDR + lo, _HDR + hi), self.backup_ranks[src],
                                               group=self._group))
                    for r in reqs:
                        r.wait()
                # confirmation: the step still in the (locked) slot after the
                # last chunk left -- 0 if it changed under the transfer
                reqs, conf = [], torch.zeros(1, dtype=torch.int64)
                if send_n:
                    ok_step = step if handler.slot_step(slot) == step else 0
                    reqs.append(dist.isend(torch.tensor([ok_step], dtype=torch.int64), self.backup_ranks[dst],
                                           group=self._group))
                if seg is not None:
                    reqs.append(dist.irecv(conf, self.backup_ranks[src], group=self._group))
                for r in reqs:
                    r.wait()
                if hdr is not None:
                    hdr[1], hdr[2] = s_n, s_m
                    if int(conf) == s_step:
                        hdr[0] = s_step
                    else:
                        logger.warning(f"replica of rank {self.backup_ranks[src]} step {s_step} discarded: "
                                       "the source slot changed during the transfer")
                    del hdr
                if seg is not None:
                    seg.close()
            return slot >= 0
        finally:
            if slot >= 0:
                self.engine._shm_locks[slot].release()

    def _replica_segment(self, peer: int, n: int, m: int) -> SharedMemory:
        name = f"replica_{peer}"
        size = _HDR + n + m
        try:
            seg = SharedMemory(name)
            if seg.size >= size:
                return seg
            seg.close()
            seg.unlink()
        except FileNotFoundError:
            pass
        return SharedMemory(name, create=True, size=size)

    # -------------------------------------------------------------- gather
    def gather(self, handler: SharedMemoryHandler):
        """Restore this rank's shm from a peer's replica if it has none
        (every member of the group calls this at restore)."""
        if not self.has_replica():
            return
        self.wait()
        with self._lock:
            self._gather(handler)

    def _gather(self, handler: SharedMemoryHandler):
        g = len(self.backup_ranks)
        have = 1 if handler.complete_step() > 0 else 0
        flags = [torch.zeros(1, dtype=torch.int64) for _ in range(g)]
        dist.all_gather(flags, torch.tensor([have], dtype=torch.int64), group=self._group)
        if all(int(f) == 1 for f in flags):
            return
        me = self._me
        for idx in range(g):
            if int(flags[idx]) == 1:
                continue
            target = self.backup_ranks[idx]
            # which live members hold a complete replica of ``target``
            holds = torch.tensor([0, 0, 0], dtype=torch.int64)
            if int(flags[me]) == 1 and idx != me:
                try:
                    seg = SharedMemory(f"replica_{target}")
                    hdr = np.frombuffer(seg.buf, dtype=np.int64, count=3)
                    holds = torch.tensor([int(hdr[0]), int(hdr[1]), int(hdr[2])], dtype=torch.int64)
                    del hdr
                    seg.close()
                except FileNotFoundError:
                    pass
            allh = [torch.zeros(3, dtype=torch.int64) for _ in range(g)]
            dist.all_gather(allh, holds, group=self._group)
            cands = [(int(h[0]), i) for i, h in enumerate(allh) if int(h[0]) > 0]
            if not cands:
                logger.warning(f"no peer holds a replica of rank {target}'s checkpoint")
                continue
            step, donor_i = max(cands, key=lambda x: (x[0], -x[1]))
            n, m = int(allh[donor_i][1]), int(allh[donor_i][2])
            donor = self.backup_ranks[donor_i]
            if me == donor_i:
                seg = SharedMemory(f"replica_{target}")
                dist.send(_u8(seg.buf, _HDR + n, _HDR + n + m), target, group=self._group)
                for lo in range(0, n, self.chunk):
                    dist.send(_u8(seg.buf, _HDR + lo, _HDR + min(n, lo + self.chunk)), target, group=self._group)
                seg.close()
            elif self.rank == target:
                mbuf = torch.empty(m, dtype=torch.uint8)
                dist.recv(mbuf, donor, group=self._group)
                meta = restricted_loads(mbuf.numpy().tobytes())
                handler.close()
                handler.init_shared_memory(create=True, size=n)
                off = handler.payload_offset(0)
                for lo in range(0, n, self.chunk):
                    dist.recv(_u8(handler.shared_memory.buf, off + lo, off + min(n, lo + self.chunk)), donor,
                              group=self._group)
                cfg = meta[DLROVER_CKPT_CONFIG_KEY]
                handler.set_meta_dict(0, meta)
                for r in range(cfg.num_slices):
                    handler.set_slice_step(0, r, cfg.step)
                logger.info(f"rank {target} restored its checkpoint shard of step {step} ({n} B) from peer {donor}")

    def close(self):
        if self._thread is not None:
            self._q.put(None)
            self._thread.join(timeout=30)
            self._thread = None
