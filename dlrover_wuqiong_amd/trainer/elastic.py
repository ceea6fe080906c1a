"""Trainer-side elasticity: fixed global batch under a changing world size,
mid-epoch resumable sampling, tunable-batch dataloader, fault injection.

Parity:
* ``ElasticTrainer``            reference dlrover/trainer/torch/elastic/trainer.py:181-336
  (grad-accumulation = max_workers*local_world / world_size, remainder on the
  low ranks; optimizer/scheduler step only on sync steps; training step
  written to runtime_metrics.json every 15 s)
* ``ElasticDistributedSampler`` elastic/sampler.py:25-158 (state_dict with the
  number of completed samples; resumes mid-epoch even if world size changed)
* ``ElasticDataLoader``         elastic/dataloader.py:26-147 (batch size from the
  parallel-config JSON written by the agent's config tuner)
"""

import contextlib
import json
import math
import os
import time
from dataclasses import dataclass
from typing import Iterator, Optional

import torch
import torch.distributed as dist
from torch.utils.data import DataLoader, Sampler

from ..atorch.fault_tolerance import heartbeat
from ..common.constants import ConfigPath, NodeEnv
from ..common.log import logger


def _rank_world():
    if dist.is_available() and dist.is_initialized():
        return dist.get_rank(), dist.get_world_size()
    return int(os.getenv("RANK", "0")), int(os.getenv("WORLD_SIZE", "1"))


def maybe_inject_fault(step: int):
    """Kill this rank at ``DWAMD_FAULT_INJECT_STEP`` on
    ``DWAMD_FAULT_INJECT_RANK`` during the first run only (restart count 0).
    ``DWAMD_FAULT_INJECT_MODE``: ``exit`` (default, exit code 17) or
    ``sigkill`` (the process is SIGKILLed: no handler, no flush, no cleanup
    -- what a crashed/OOM-killed rank looks like to the agent).
    Used by the goodput benchmark and the agent tests."""
    s = os.getenv(NodeEnv.FAULT_INJECT_STEP, "")
    if not s or int(os.getenv("TORCHELASTIC_RESTART_COUNT", "0")) != 0:
        return
    r = int(os.getenv(NodeEnv.FAULT_INJECT_RANK, "0"))
    if step == int(s) and _rank_world()[0] == r:
        logger.error(f"injected fault at step {step} on rank {r}")
        if os.getenv("DWAMD_FAULT_INJECT_MODE", "exit") == "sigkill":
            import signal

            os.kill(os.getpid(), signal.SIGKILL)
        os._exit(17)


def standby_point(prepin_shm: bool = True):
    """Deep warm-standby hand-off (see ``elastic_agent/standby.py``): call
    after world-independent set-up (device, model, optimizer, warm-up) and
    before ``init_process_group``.  Returns ``None`` when this process is a
    regular worker, activation info when it was a standby."""
    from ..elastic_agent.standby import standby_point as _sp

    return _sp(prepin_shm=prepin_shm)


def training_stream(device=None) -> "torch.cuda.Stream":
    """The stream to train on: the current stream when it is not the
    device's default one (an import standby made the stream its HBM
    reservation belongs to current -- allocations on it reuse the
    reservation instead of asking the driver for fresh VRAM right after a
    restart), else a new non-blocking stream.  Callers set it current."""
    dev = torch.device("cuda", torch.cuda.current_device()) if device is None else torch.device(device)
    cur = torch.cuda.current_stream(dev)
    if cur != torch.cuda.default_stream(dev):
        return cur
    return torch.cuda.Stream(dev)


@dataclass
class GradientState:
    num_steps: int = 0
    num_backward_steps: int = 0
    sync_gradients: bool = True

    def check_sync_gradient(self, accum: int):
        self.sync_gradients = self.num_backward_steps % max(1, accum) == 0


class _ElasticOptimizer:
    """Steps the wrapped optimizer only on gradient-sync steps."""

    def __init__(self, optimizer, trainer):
        self.optimizer = optimizer
        self._trainer = trainer

    def step(self, *a, **kw):
        if self._trainer.gradient_state.sync_gradients:
            return self.optimizer.step(*a, **kw)

    def zero_grad(self, *a, **kw):
        if self._trainer.gradient_state.sync_gradients:
            return self.optimizer.zero_grad(*a, **kw)

    def __getattr__(self, name):
        return getattr(self.optimizer, name)


class _ElasticLRScheduler:
    def __init__(self, scheduler, trainer):
        self.scheduler = scheduler
        self._trainer = trainer

    def step(self, *a, **kw):
        if self._trainer.gradient_state.sync_gradients:
            return self.scheduler.step(*a, **kw)

    def __getattr__(self, name):
        return getattr(self.scheduler, name)


class ElasticTrainer:
    def __init__(self, model, dataloader=None, report_interval: float = 15.0):
        self.model = model
        self.dataloader = dataloader
        self.gradient_state = GradientState()
        self.gradient_accumulation_steps = 1
        self._report_interval = report_interval
        self._last_report = 0.0
        from ..utils.xpu_timer import maybe_install_from_env

        maybe_install_from_env()

    def prepare(self, optimizer, lr_scheduler=None):
        self._set_gradient_accumulation_steps()
        opt = _ElasticOptimizer(optimizer, self)
        if lr_scheduler is not None:
            return opt, _ElasticLRScheduler(lr_scheduler, self)
        return opt

    def _set_gradient_accumulation_steps(self):
        max_workers = int(os.getenv(NodeEnv.WORKER_NUM, os.getenv(NodeEnv.NODE_NUM, "1")) or 1)
        local = int(os.getenv("LOCAL_WORLD_SIZE", "1"))
        target = max(1, max_workers) * local
        rank, world = _rank_world()
        self.gradient_accumulation_steps = max(1, target // world)
        if rank < target % world:
            self.gradient_accumulation_steps += 1
        logger.info(f"rank {rank}/{world}: gradient accumulation steps {self.gradient_accumulation_steps}")

    @contextlib.contextmanager
    def step(self, fix_total_batch_size: bool = False):
        gs = self.gradient_state
        gs.num_backward_steps += 1
        if fix_total_batch_size:
            gs.check_sync_gradient(self.gradient_accumulation_steps)
        else:
            gs.sync_gradients = True
        ctx = contextlib.nullcontext
        if not gs.sync_gradients:
            ctx = getattr(self.model, "no_sync", ctx)
        with ctx():
            yield
        if gs.sync_gradients:
            gs.num_steps += 1
            heartbeat()
            maybe_inject_fault(gs.num_steps)
            now = time.time()
            if now - self._last_report > self._report_interval:
                self.report_training_step()
                self._last_report = now
        if isinstance(self.dataloader, ElasticDataLoader):
            self.dataloader.update_batch_size()

    @property
    def num_steps(self):
        return self.gradient_state.num_steps

    def reset(self):
        self.gradient_state.num_steps = 0

    def report_training_step(self):
        path = os.getenv(ConfigPath.ENV_RUNTIME_METRICS, ConfigPath.RUNTIME_METRICS)
        rank, _ = _rank_world()
        if rank != 0:
            return
        try:
            os.makedirs(os.path.dirname(path), exist_ok=True)
            tmp = path + ".tmp"
            with open(tmp, "w") as f:
                json.dump({"step": self.gradient_state.num_steps, "timestamp": time.time()}, f)
            os.replace(tmp, path)
        except OSError:
            pass


class ElasticDistributedSampler(Sampler):
    """Deterministic per-epoch shuffle; ``state_dict`` records how many
    samples the whole job completed, so after a restart with a different
    world size every rank resumes from exactly the next unseen sample."""

    def __init__(self, dataset, num_replicas: Optional[int] = None, rank: Optional[int] = None,
                 shuffle: bool = True, seed: int = 0, drop_last: bool = False):
        r, w = _rank_world()
        self.dataset = dataset
        self.num_replicas = num_replicas if num_replicas is not None else w
        self.rank = rank if rank is not None else r
        self.shuffle = shuffle
        self.seed = seed
        self.drop_last = drop_last
        self.epoch = 0
        self.completed_num = 0
        self._update_sizes()

    def _update_sizes(self):
        n = len(self.dataset) - self.completed_num
        if self.drop_last and n % self.num_replicas:
            self.num_samples = n // self.num_replicas
        else:
            self.num_samples = math.ceil(n / self.num_replicas)
        self.total_size = self.num_samples * self.num_replicas

    def __iter__(self) -> Iterator[int]:
        if self.shuffle:
            g = torch.Generator()
            g.manual_seed(self.seed + self.epoch)
            idx = torch.randperm(len(self.dataset), generator=g).tolist()
        else:
            idx = list(range(len(self.dataset)))
        idx = idx[self.completed_num:]
        self._update_sizes()
        if not self.drop_last:
            pad = self.total_size - len(idx)
            if pad > 0:
                idx += (idx * math.ceil(pad / max(1, len(idx))))[:pad]
        else:
            idx = idx[: self.total_size]
        return iter(idx[self.rank: self.total_size: self.num_replicas])

    def __len__(self):
        return self.num_samples

    def set_epoch(self, epoch: int):
        if epoch != self.epoch:
            self.completed_num = 0
        self.epoch = epoch

    def state_dict(self, iter_step: int, micro_batch_size: int) -> dict:
        """``iter_step`` local steps of ``micro_batch_size`` completed."""
        done = self.completed_num + iter_step * micro_batch_size * self.num_replicas
        return {"epoch": self.epoch, "completed_num": min(done, len(self.dataset))}

    def load_state_dict(self, state: dict):
        self.epoch = int(state.get("epoch", 0))
        self.completed_num = int(state.get("completed_num", 0))
        self._update_sizes()


class ElasticDataLoader(DataLoader):
    """DataLoader whose batch size follows the agent's parallel-config file
    (``DLROVER_PARAL_CONFIG_PATH``), enabling batch-size auto-tuning."""

    def __init__(self, *args, config_file: str = "", **kwargs):
        super().__init__(*args, **kwargs)
        self.config_file = config_file or os.getenv(ConfigPath.ENV_PARAL_CONFIG, ConfigPath.PARAL_CONFIG)
        self._version = 0
        self.load_config()

    def load_config(self):
        try:
            with open(self.config_file) as f:
                cfg = json.load(f)
        except (OSError, ValueError):
            return
        dl = cfg.get("dataloader", {})
        v = int(dl.get("version", 0))
        bs = int(dl.get("batch_size", 0))
        if v > self._version and bs > 0 and self.batch_sampler is not None:
            self.batch_sampler.batch_size = bs
            self._version = v
            logger.info(f"ElasticDataLoader: batch size -> {bs} (config v{v})")

    def update_batch_size(self, batch_size: int = 0):
        if batch_size > 0 and self.batch_sampler is not None:
            self.batch_sampler.batch_size = batch_size
        else:
            self.load_config()
