"""Agent-side asynchronous checkpoint persister.

Lives in the (long-lived) agent process, or in a daemon thread of local rank 0
when training runs without the agent.  Workers tell it *which* saver class to
build through the ``factory`` queue (a :class:`ClassMeta`), then send
``CheckpointEvent``s on the event queue.  For every SAVE event it persists
each local shard from shm to storage (one thread per shard), writes a done
file per shard, and node 0 commits the step (tracker file) once every global
shard is done.  On SIGTERM / worker failure the latest complete in-memory
checkpoint is persisted ("save at breakpoint").

Parity: reference ``dlrover/python/elastic_agent/torch/ckpt_saver.py``
(``AsyncCheckpointSaver`` :344-771, ``CommonDirCheckpointSaver`` :773,
``TempDirCheckpointSaver`` :924, ``DdpCheckpointSaver`` :1117,
``MegatronCheckpointSaver`` :1127, ``DeepSpeedCheckpointSaver`` :1145,
``FsdpDcpSaver`` :1165).
"""

import os
import queue as pyqueue
import signal
import threading
import time
from concurrent.futures import ThreadPoolExecutor
from typing import List, Optional

import torch

from ..common import env_utils
from ..common.constants import CheckpointConstant
from ..common.log import logger
from ..common.multi_process import SharedLock, SharedQueue
from ..common.serialize import ClassMeta
from ..flash_checkpoint.engine import CheckpointEvent, CheckpointEventType
from ..flash_checkpoint.shm_handler import (DLROVER_CKPT_CONFIG_KEY, EVENT_QUEUE_SIZE, CheckpointConfig,
                                            CheckpointSharedObjPrefix, SharedMemoryHandler, slot_lock_name)


def _writer_for(path: str):
    """File format by extension: safetensors for ``*.safetensors`` (HF
    weights), a ``torch.save`` archive otherwise -- written by
    :func:`fast_torch_save` (storages streamed from shm with parallel pwrite;
    ``DWAMD_PERSIST_WRITER=torch`` selects plain ``torch.save``)."""
    if str(path).endswith(".safetensors"):
        def write(sd, p):
            from safetensors.torch import save_file

            save_file({k: v.contiguous() for k, v in sd.items()}, p, metadata={"format": "pt"})

        return write
    if os.environ.get("DWAMD_PERSIST_WRITER", "fast") == "torch":
        return torch.save
    from ..common.storage import fast_torch_save

    threads = int(os.environ.get("DWAMD_PERSIST_THREADS", "16"))
    return lambda sd, p: fast_torch_save(sd, p, threads=threads)


class AsyncCheckpointSaver:
    _saver_instance: Optional["AsyncCheckpointSaver"] = None
    _factory_started = False
    _STAGE_DIR = "._dlrover_ckpt_stage"

    def __init__(self, checkpoint_dir, storage_meta: ClassMeta, local_shard_num=1, global_shard_num=1,
                 save_timeout=CheckpointConstant.SAVE_TIMEOUT):
        self.checkpoint_dir = checkpoint_dir
        self.local_shard_num = local_shard_num
        self.global_shard_num = global_shard_num
        self._node_rank = env_utils.get_node_rank()
        self._is_agent_rank_0 = self._node_rank == 0
        self._save_timeout = save_timeout
        self.storage = storage_meta.build()
        self._writing_storage = False
        self._latest_step = 0
        self._stop_commit = False
        self._closed = False
        self._event_queue = SharedQueue(CheckpointSharedObjPrefix.SAVE_STEP_QNAME + "0", create=True,
                                        maxsize=EVENT_QUEUE_SIZE)
        self._shm_handlers: List[SharedMemoryHandler] = []
        self._shm_locks: List[List[SharedLock]] = []  # [shard][slot]
        for i in range(local_shard_num):
            h = SharedMemoryHandler(i, host=True)
            self._shm_handlers.append(h)
            self._shm_locks.append([SharedLock(slot_lock_name(i, s), create=True) for s in range(h.num_slots)])
        self._executor = ThreadPoolExecutor(max_workers=max(1, local_shard_num), thread_name_prefix="ckpt_saver")
        self.last_persist_sec = 0.0
        logger.info(f"{type(self).__name__}: dir={checkpoint_dir} local_shards={local_shard_num} "
                    f"global_shards={global_shard_num}")

    # ------------------------------------------------------------ lifecycle
    @classmethod
    def start_async_saving_ckpt(cls):
        """Start the factory thread that builds the saver requested by the
        training processes and runs its event loop."""
        from ..common.multi_process import shm_name

        ns = shm_name("", "")
        if cls._factory_started == ns:
            return
        cls._factory_started = ns
        fq = SharedQueue("factory", create=True, maxsize=4)

        def run_saver(meta: ClassMeta):
            if cls._saver_instance is not None:
                cls._saver_instance.close()
            saver = meta.build()
            cls._saver_instance = saver
            saver._sync_shm_to_storage()

        def factory():
            thread = None
            while True:
                try:
                    meta = fq.get()
                except Exception:  # pragma: no cover
                    time.sleep(0.5)
                    continue
                if cls._saver_instance is not None and thread is not None and thread.is_alive():
                    cur = cls._saver_instance
                    if (cur.checkpoint_dir == meta.kwargs.get("checkpoint_dir")
                            and type(cur).__name__ == meta.class_name):
                        continue
                thread = threading.Thread(target=run_saver, args=(meta,), daemon=True, name="checkpoint-saver")
                thread.start()

        threading.Thread(target=factory, daemon=True, name="checkpoint-saver-factory").start()

    @classmethod
    def get_ckpt_saver(cls):
        return cls._saver_instance

    @classmethod
    def register_signal_handler(cls):
        prev_int = signal.getsignal(signal.SIGINT)
        prev_term = signal.getsignal(signal.SIGTERM)

        def chain(prev, signum, frame):
            if callable(prev):
                prev(signum, frame)
            elif prev != signal.SIG_IGN:
                # default disposition: terminate (via SystemExit so that the
                # launcher's cleanup/finally blocks still run)
                raise SystemExit(128 + signum)

        def on_int(signum, frame):
            if cls._saver_instance:
                cls._saver_instance.close()
            chain(prev_int, signum, frame)

        def on_term(signum, frame):
            if cls._saver_instance:
                try:
                    cls._saver_instance.save_shm_to_storage()
                finally:
                    cls._saver_instance.close()
            chain(prev_term, signum, frame)

        signal.signal(signal.SIGINT, on_int)
        signal.signal(signal.SIGTERM, on_term)

    @classmethod
    def reset(cls):
        if cls._saver_instance is not None:
            cls._saver_instance.reset_shared_memory()

    def reset_shared_memory(self):
        # workers restart: re-attach lazily (only if a segment was re-created);
        # an in-flight breakpoint persist keeps running
        for h in self._shm_handlers:
            h.reset()

    def wait_saving_checkpoint(self):
        return self._writing_storage

    def close(self):
        if self._closed:
            return
        self._closed = True
        try:
            self._event_queue.put(CheckpointEvent(type=CheckpointEventType.EXIT), block=False)
        except Exception:
            pass
        for h in self._shm_handlers:
            h.close()
        self._executor.shutdown(wait=False)

    def unlink_all(self):
        for h in self._shm_handlers:
            h.unlink()
        for locks in self._shm_locks:
            for lk in locks:
                lk.unlink()
        self._event_queue.unlink()

    # ------------------------------------------------------------- loop
    def _sync_shm_to_storage(self):
        logger.info("async flash-checkpoint saver started")
        while not self._closed:
            try:
                ev: CheckpointEvent = self._event_queue.get(timeout=1.0)
            except pyqueue.Empty:
                continue
            if ev.type == CheckpointEventType.UPDATE_SHARD:
                self.global_shard_num = ev.global_shard_num
            elif ev.type == CheckpointEventType.SAVE:
                try:
                    self.save_step_checkpoint(ev.step)
                except Exception as e:  # keep the loop alive
                    logger.error(f"persisting step {ev.step} failed: {e}", exc_info=True)
            elif ev.type == CheckpointEventType.EXIT:
                break

    # ---------------------------------------------------------- persisting
    def _get_checkpoint_done_dir(self, step):
        return os.path.join(self.checkpoint_dir, self._STAGE_DIR, f"{step}.done")

    def _wait_shard_complete(self, handler: SharedMemoryHandler, step: int, timeout: float) -> int:
        """Slot holding ``step`` complete, or -1 (timeout / overwritten by a newer step)."""
        deadline = time.time() + timeout
        while time.time() < deadline:
            steps = handler.complete_steps()
            if step in steps:
                return steps[step]
            if steps and min(steps) > step:
                return -1
            time.sleep(0.01)
        return -1

    def _save_shard(self, step: int, shard_id: int, done_dir: str) -> bool:
        h = self._shm_handlers[shard_id]
        slot = self._wait_shard_complete(h, step, self._save_timeout)
        if slot < 0:
            logger.error(f"shard {shard_id} does not hold a complete step {step}")
            return False
        lock = self._shm_locks[shard_id][slot]
        if not lock.acquire(blocking=True, timeout=self._save_timeout):
            return False
        try:
            if h.slot_step(slot) != step:
                logger.error(f"shard {shard_id}: slot {slot} was overwritten before step {step} was persisted")
                return False
            cfg = h.get_checkpoint_config(slot=slot)
            self.persist_to_storage(shard_id, cfg, slot)
        finally:
            lock.release()
        self.storage.write("done", os.path.join(done_dir, str(cfg.rank)))
        return True

    def save_step_checkpoint(self, step: int):
        self._writing_storage = True
        t0 = time.time()
        try:
            done_dir = self._get_checkpoint_done_dir(step)
            self.storage.safe_makedirs(done_dir)
            futs = [self._executor.submit(self._save_shard, step, i, done_dir) for i in range(self.local_shard_num)]
            ok = all(f.result() for f in futs)
            if ok and self._is_agent_rank_0:
                self.commit_checkpoint(step, done_dir, self._save_timeout)
            self._latest_step = max(self._latest_step, step) if ok else self._latest_step
            self.last_persist_sec = time.time() - t0
            logger.info(f"persisted step {step} in {self.last_persist_sec:.2f}s (ok={ok})")
        finally:
            self._writing_storage = False

    def persist_to_storage(self, shard_id: int, cfg: CheckpointConfig, slot: int):
        """Write each category of the shard's state dict to its path."""
        h = self._shm_handlers[shard_id]
        sd = h.load_state_dict(slot)
        sd.pop(DLROVER_CKPT_CONFIG_KEY, None)
        for name, path in (cfg.paths or {}).items():
            if name in sd:
                self.storage.write_state_dict(sd[name], path, _writer_for(path))

    def commit_checkpoint(self, step: int, step_done_dir: str, timeout=600):
        deadline = time.time() + timeout
        while time.time() < deadline:
            if self._stop_commit:
                self._stop_commit = False
                return False
            n = len(self.storage.listdir(step_done_dir)) if self.storage.exists(step_done_dir) else 0
            if n >= self.global_shard_num:
                if not self._finalize_step(step):
                    self.storage.commit(step, False)
                    return False
                self.update_tracker_file(step)
                self.storage.safe_rmtree(step_done_dir)
                self.storage.commit(step, True)
                return True
            time.sleep(0.2)
        logger.error(f"commit of step {step} timed out")
        self.storage.commit(step, False)
        return False

    def _finalize_step(self, step: int) -> bool:
        """Hook run on node 0 once every global shard is on storage."""
        return True

    def update_tracker_file(self, step: int):
        self.storage.write(str(step), os.path.join(self.checkpoint_dir, CheckpointConstant.TRACER_FILE_NAME))

    # ------------------------------------------------------ breakpoint save
    def save_shm_to_storage(self, timeout: int = 60, master_client=None):
        """Persist the latest complete in-memory checkpoint (e.g. after a
        worker failure, before restarting the workers)."""
        common = None
        per_shard = []
        for h in self._shm_handlers:
            steps = set(h.complete_steps())
            per_shard.append(sorted(steps))
            common = steps if common is None else common & steps
        logger.info(f"breakpoint save: complete in-memory steps per local shard: {per_shard}")
        if not common:
            logger.info("no complete in-memory checkpoint to persist")
            return False
        step = max(common)
        if master_client is not None and not self._sync_node_checkpoint(master_client, step, timeout):
            self._stop_commit = True
            return False
        busy = any(locks[h.slot_of(step)].locked() for h, locks in zip(self._shm_handlers, self._shm_locks)
                   if h.slot_of(step) >= 0)
        if self._writing_storage or busy:
            logger.info("saver busy; skip breakpoint save")
            return False
        if step > self._latest_step:
            self.save_step_checkpoint(step)
            return True
        return False

    def _sync_node_checkpoint(self, master_client, step, timeout):
        deadline = time.time() + timeout
        while time.time() < deadline:
            if master_client.sync_checkpoint(step):
                return True
            time.sleep(1)
        return False


class CommonDirCheckpointSaver(AsyncCheckpointSaver):
    """Persist each shard straight to the user path (framework-chosen)."""


class TempDirCheckpointSaver(AsyncCheckpointSaver):
    """Persist into a staging dir, then move into place at commit."""

    def persist_to_storage(self, shard_id, cfg, slot):
        h = self._shm_handlers[shard_id]
        sd = h.load_state_dict(slot)
        sd.pop(DLROVER_CKPT_CONFIG_KEY, None)
        stage = os.path.join(self.checkpoint_dir, self._STAGE_DIR, str(cfg.step))
        for name, path in (cfg.paths or {}).items():
            if name in sd:
                rel = os.path.relpath(path, self.checkpoint_dir)
                self.storage.write_state_dict(sd[name], os.path.join(stage, rel), _writer_for(path))

    def commit_checkpoint(self, step, step_done_dir, timeout=600):
        stage = os.path.join(self.checkpoint_dir, self._STAGE_DIR, str(step))
        deadline = time.time() + timeout
        while time.time() < deadline:
            n = len(self.storage.listdir(step_done_dir)) if self.storage.exists(step_done_dir) else 0
            if n >= self.global_shard_num:
                for root, _dirs, files in os.walk(stage):
                    for f in files:
                        src = os.path.join(root, f)
                        dst = os.path.join(self.checkpoint_dir, os.path.relpath(src, stage))
                        os.makedirs(os.path.dirname(dst), exist_ok=True)
                        os.replace(src, dst)
                self.storage.safe_rmtree(stage)
                self.update_tracker_file(step)
                self.storage.safe_rmtree(step_done_dir)
                self.storage.commit(step, True)
                return True
            time.sleep(0.2)
        self.storage.commit(step, False)
        return False


class DdpCheckpointSaver(CommonDirCheckpointSaver):
    """DDP: only node 0 holds the shard that is written (replicated state)."""

    def save_step_checkpoint(self, step):
        if self._node_rank != 0:
            return
        super().save_step_checkpoint(step)


class MegatronCheckpointSaver(CommonDirCheckpointSaver):
    TRACER_FILE = "latest_checkpointed_iteration.txt"

    def update_tracker_file(self, step):
        super().update_tracker_file(step)
        self.storage.write(str(step), os.path.join(self.checkpoint_dir, self.TRACER_FILE))


class DeepSpeedCheckpointSaver(CommonDirCheckpointSaver):
    """Commits DeepSpeed's ``latest`` with the checkpoint's tag (free-form,
    e.g. ``global_step100``); ``._dlrover_ds_tags/{step}`` remembers it so a
    later memory-only save can restore ``latest``."""

    TRACER_FILE = "latest"
    TAGS_DIR = "._dlrover_ds_tags"

    def persist_to_storage(self, shard_id, cfg, slot):
        super().persist_to_storage(shard_id, cfg, slot)
        tag = (cfg.paths or {}).get("__tag__")
        if tag:
            if not hasattr(self, "_step_tags"):
                self._step_tags = {}
            self._step_tags[cfg.step] = tag

    def update_tracker_file(self, step):
        super().update_tracker_file(step)
        tag = getattr(self, "_step_tags", {}).pop(step, str(step))
        self.storage.write(tag, os.path.join(self.checkpoint_dir, self.TAGS_DIR, str(step)))
        self.storage.write(tag, os.path.join(self.checkpoint_dir, self.TRACER_FILE))


class FsdpFlatCheckpointSaver(TempDirCheckpointSaver):
    """ATorch flat FSDP layout (atorch/fsdp_flat_ckpt.py): tensor categories
    as safetensors streamed from shm, metadata as JSON, staged then moved
    into place; tracker ``latest_checkpointed_iteration.txt``.  Parity:
    reference atorch/atorch/utils/fsdp_async_ckpt_util.py:29-67."""

    TRACER_FILE = "latest_checkpointed_iteration.txt"

    def persist_to_storage(self, shard_id, cfg, slot):
        import json

        from ..atorch.fsdp_flat_ckpt import BUFFERS, CKPT_META, OPTIM_STATES, PARAM_GROUPS, PARAM_META, PARAMS
        from ..atorch.fsdp_flat_ckpt import safetensors_dump

        h = self._shm_handlers[shard_id]
        sd = h.load_state_dict(slot)
        sd.pop(DLROVER_CKPT_CONFIG_KEY, None)
        stage = os.path.join(self.checkpoint_dir, self._STAGE_DIR, str(cfg.step))
        for name, path in (cfg.paths or {}).items():
            if name not in sd:
                continue
            dst = os.path.join(stage, os.path.relpath(path, self.checkpoint_dir))
            if name in (PARAMS, OPTIM_STATES, BUFFERS):
                safetensors_dump(sd[name], dst)
            elif name in (PARAM_META, PARAM_GROUPS, CKPT_META):
                os.makedirs(os.path.dirname(dst), exist_ok=True)
                with open(dst, "w") as f:
                    json.dump(sd[name], f)
            else:
                self.storage.write_state_dict(sd[name], dst, _writer_for(path))

    def update_tracker_file(self, step):
        super().update_tracker_file(step)
        self.storage.write(str(step), os.path.join(self.checkpoint_dir, self.TRACER_FILE))


class FsdpDcpSaver(CommonDirCheckpointSaver):
    """Writes torch.distributed.checkpoint-compatible ``.distcp`` shards +
    ``.metadata`` (see flash_checkpoint/fsdp.py for the layout)."""

    def persist_to_storage(self, shard_id, cfg, slot):
        from ..flash_checkpoint.fsdp import persist_dcp_shard

        h = self._shm_handlers[shard_id]
        sd = h.load_state_dict(slot)
        sd.pop(DLROVER_CKPT_CONFIG_KEY, None)
        path = persist_dcp_shard(self.storage, sd, cfg)
        if not hasattr(self, "_step_paths"):
            self._step_paths = {}
        self._step_paths[cfg.step] = (path, cfg.world_size)

    def _finalize_step(self, step):
        from ..flash_checkpoint.fsdp import finalize_dcp_checkpoint

        path, world = getattr(self, "_step_paths", {}).pop(step, (None, 0))
        if path is None:
            logger.error(f"no DCP path recorded for step {step}")
            return False
        return finalize_dcp_checkpoint(self.storage, path, world)
