"""AtorchTrainer: a HuggingFace-``Trainer``-compatible training loop whose
model / optimizer / data pipeline come from ``auto_accelerate`` and whose
checkpoints go through the flash-checkpoint engine.

    args = AtorchTrainingArgs(output_dir="out", max_steps=1000, save_steps=100,
                              atorch_opt="fsdp", atorch_wrap_cls=(LlamaDecoderLayer,),
                              bf16=True, flash_checkpoint=True)
    trainer = AtorchTrainer(model, args, train_dataset=ds, data_collator=collate)
    trainer.train(resume_from_checkpoint=True)

What it does (same contract as the reference, MI355X-first internals):

* ``_atorch_init`` builds the load strategy from the arguments
  (``atorch_opt`` = ddp | fsdp | zero2 | zero1, ``atorch_wrap_cls``,
  ``atorch_checkpoint_cls`` for activation checkpointing, bf16/fp16 autocast,
  ``atorch_module_replace`` for the fused HIP norms) and calls
  ``auto_accelerate`` -> model, optimizer, distributed dataloader;
* the loop does gradient accumulation (``no_sync`` on all but the last
  micro-step), grad-norm clipping, LR scheduling (transformers'
  ``get_scheduler``), logging, periodic evaluation and HF ``TrainerCallback``
  events (``on_step_end`` / ``on_log`` / ``on_save`` ...);
* ``save_steps``: with ``flash_checkpoint=True`` the model + optimizer +
  scheduler + RNG state is snapshotted to host shm in the training pause and
  persisted asynchronously (``DdpCheckpointer`` / ``FsdpShardCheckpointer``);
  otherwise written synchronously.  ``trainer_state.json`` is written by rank
  0 next to it, and ``save_total_limit`` rotates old checkpoints;
* ``resume_from_checkpoint`` (path or True = latest) restores everything,
  preferring the in-memory copy after an in-place restart, and skips the
  already-consumed batches of the current epoch.

Parity: ATorch ``atorch/trainer/atorch_trainer.py`` (``AtorchTrainer``:
``train`` :666, ``_inner_training_loop`` :717, ``_save_checkpoint`` :1304,
``_rotate_checkpoints`` :1714, ``evaluate`` :1742, ``predict`` :1801,
``training_step`` :2043, ``compute_loss`` :2196) and
``atorch/trainer/atorch_args.py`` (``AtorchArguments``).
"""

import json
import math
import os
import random
import re
import shutil
import time
from dataclasses import dataclass, field
from typing import Any, Callable, Dict, List, NamedTuple, Optional, Tuple

import numpy as np
import torch
import torch.distributed as dist
import torch.nn as nn

from ..common.log import logger
from ..common.serialize import safe_torch_load

try:
    from transformers import TrainingArguments
    from transformers.trainer_callback import (CallbackHandler, DefaultFlowCallback, PrinterCallback, TrainerControl,
                                               TrainerState)
except ImportError as e:  # pragma: no cover
    raise ImportError("AtorchTrainer needs transformers") from e

PREFIX_CHECKPOINT_DIR = "checkpoint"
TRAINER_STATE_NAME = "trainer_state.json"
STATE_FILE = "atorch_state.pt"


@dataclass
class AtorchTrainingArgs(TrainingArguments):
    atorch_opt: str = field(default="ddp", metadata={"help": "ddp | fsdp | zero2 | zero1 | none"})
    atorch_parallel_mode: bool = field(default=True, metadata={"help": "create named parallel groups"})
    atorch_module_replace: bool = field(default=True, metadata={"help": "fused HIP norms"})
    atorch_wrap_cls: Optional[Tuple[Any, ...]] = field(default=None, metadata={"help": "FSDP wrap classes"})
    atorch_checkpoint_cls: Optional[Tuple[Any, ...]] = field(default=None,
                                                             metadata={"help": "activation checkpoint classes"})
    load_strategy: Optional[List[Any]] = field(default=None, metadata={"help": "explicit auto_accelerate strategy"})
    optim_func: Optional[Callable] = field(default=None, metadata={"help": "optimizer class"})
    optim_args: Optional[Dict] = field(default=None, metadata={"help": "optimizer kwargs"})
    optim_param_func: Optional[Callable] = field(default=None, metadata={"help": "model -> param groups"})
    loss_func: Optional[Callable] = field(default=None, metadata={"help": "(batch, output) -> loss"})
    prepare_input: Optional[Callable] = field(default=None, metadata={"help": "(batch, device) -> batch"})
    model_input_format: Optional[str] = field(default="unpack_dict",
                                              metadata={"help": "unpack_dict | unpack_sequence | None"})
    flash_checkpoint: bool = field(default=True, metadata={"help": "save through the flash-checkpoint engine"})
    async_save: bool = field(default=True, metadata={"help": "persist flash checkpoints asynchronously"})
    shuffle: bool = field(default=True, metadata={"help": "shuffle the training data"})
    skip_if_nonfinite: bool = field(default=True, metadata={"help": "skip steps with non-finite grad norm"})
    # the rest of the reference's AtorchArguments (trainer/atorch_args.py:21-190)
    ignore_dryrun_on_load_strategy: bool = field(default=True, metadata={"help": "no dry run of a loaded strategy"})
    save_load_by_streaming: bool = field(default=False, metadata={"help": "accepted; saves stream through the "
                                                                          "flash-checkpoint engine anyway"})
    save_base_model: bool = field(default=False, metadata={"help": "PEFT: also save the base model"})
    use_atorch_dataloader: bool = field(default=True, metadata={"help": "dataloader built by auto_accelerate"})
    distributed_sampler_cls: Optional[Callable] = field(default=None, metadata={"help": "custom sampler class"})
    excluded: Optional[List[str]] = field(default=None, metadata={"help": "optimizations never used"})
    included: Optional[List[str]] = field(default=None, metadata={"help": "optimizations always used"})
    finetune_strategy: bool = field(default=False, metadata={"help": "accepted (no strategy search on load)"})
    save_strategy_to_file: Optional[str] = field(default=None, metadata={"help": "write the strategy as JSON"})
    use_default_data_collator: bool = field(default=False, metadata={"help": "pad batches with "
                                                                              "DataCollatorWithPadding"})
    ignore_write_errors: bool = field(default=False, metadata={"help": "log and continue on checkpoint write errors"})
    atorch_lr_scheduler_type: Optional[str] = field(default=None, metadata={"help": "overrides lr_scheduler_type"})
    cpu_offload: bool = field(default=False, metadata={"help": "FSDP: parameters / optimizer state on the host"})
    use_orig_params: bool = field(default=True, metadata={"help": "FSDP2 always keeps the original parameters"})
    wrap_trainable_outmost: bool = field(default=False, metadata={"help": "accepted"})
    sync_module_states: bool = field(default=True, metadata={"help": "FSDP: broadcast rank 0's initial weights"})
    limit_all_gathers: bool = field(default=True, metadata={"help": "accepted (FSDP2 bounds all-gathers itself)"})
    forward_prefetch: bool = field(default=True, metadata={"help": "accepted (FSDP2 prefetches the next layer)"})
    max_shard_size: str = field(default="10GB", metadata={"help": "save_pretrained shard size"})
    logit_names: Optional[List[str]] = field(default=None, metadata={"help": "output keys holding the logits"})
    logit_index: int = field(default=-1, metadata={"help": "tuple-output index of the logits"})

    def __post_init__(self):
        if not self.report_to:
            self.report_to = []
        super().__post_init__()


class TrainResult(NamedTuple):
    """HF ``TrainOutput`` (``.global_step``, ``.training_loss``, ``.metrics``)
    that also answers ``result["train_loss"]`` / ``result["global_step"]``."""

    global_step: int
    training_loss: float
    metrics: Dict[str, Any]

    def __getitem__(self, k):
        if isinstance(k, str):
            return self.metrics[k]
        return tuple.__getitem__(self, k)


def _count_params(model: nn.Module) -> Tuple[int, int]:
    total = sum(p.numel() for p in model.parameters())
    train = sum(p.numel() for p in model.parameters() if p.requires_grad)
    return total, train


class AtorchTrainer:
    def __init__(self, model: nn.Module, args: AtorchTrainingArgs, data_collator=None, train_dataset=None,
                 eval_dataset=None, tokenizer=None, compute_metrics=None, callbacks=None, optimizers=(None, None),
                 preprocess_logits_for_metrics=None):
        self.args = args
        # (logits, labels) -> what compute_metrics needs, applied per eval
        # batch on the device (reference atorch_trainer.py:149)
        self.preprocess_logits_for_metrics = preprocess_logits_for_metrics
        self.data_collator = data_collator
        self.train_dataset = train_dataset
        self.eval_dataset = eval_dataset
        self.tokenizer = tokenizer
        self.compute_metrics = compute_metrics
        self.model, self.optimizer, self.lr_scheduler = model, optimizers[0], optimizers[1]
        self.train_dataloader = None
        self.strategy = None
        self.device = torch.device("cpu")
        self.amp_dtype = None
        self._checkpointer = None
        self._atorch_init()
        cbs = [DefaultFlowCallback] + (callbacks or [])
        if not args.disable_tqdm:
            cbs.append(PrinterCallback)
        self.callback_handler = CallbackHandler(cbs, self.model, tokenizer, self.optimizer, self.lr_scheduler)
        self.state = TrainerState()
        self.control = TrainerControl()
        os.makedirs(args.output_dir, exist_ok=True)

    # ---------------------------------------------------------------- setup
    def _rank(self) -> int:
        return dist.get_rank() if dist.is_initialized() else 0

    def _world(self) -> int:
        return dist.get_world_size() if dist.is_initialized() else 1

    def is_world_process_zero(self) -> bool:
        return self._rank() == 0

    def is_local_process_zero(self) -> bool:
        return int(os.environ.get("LOCAL_RANK", "0")) == 0

    def add_callback(self, cb):
        self.callback_handler.add_callback(cb)

    def pop_callback(self, cb):
        return self.callback_handler.pop_callback(cb)

    def _build_strategy(self):
        a = self.args
        if a.load_strategy is not None:
            return a.load_strategy
        s: List[Any] = []
        if a.atorch_parallel_mode:
            s.append("parallel_mode")
        if a.atorch_module_replace:
            s.append("module_replace")
        if a.bf16 or a.fp16:
            s.append(("amp_native", {"dtype": torch.bfloat16 if a.bf16 else torch.float16}))
        if a.atorch_checkpoint_cls:
            s.append(("checkpoint", {"wrap_cls": tuple(a.atorch_checkpoint_cls)}))
        opt = (a.atorch_opt or "none").lower()
        if opt in ("fsdp", "zero2"):
            cfg = {"sync_module_states": a.sync_module_states, "use_orig_params": a.use_orig_params,
                   "limit_all_gathers": a.limit_all_gathers, "forward_prefetch": a.forward_prefetch,
                   "cpu_offload": a.cpu_offload}
            if a.atorch_wrap_cls:
                cfg["wrap_cls"] = tuple(a.atorch_wrap_cls)
            s.append((opt, cfg))
        elif opt in ("zero1", "ddp"):
            s.append(opt)
        return s

    def _atorch_init(self):
        from .auto_accelerate import auto_accelerate

        a = self.args
        optim_func = a.optim_func
        optim_args = dict(a.optim_args or {})
        if self.optimizer is None and optim_func is None:
            optim_func = torch.optim.AdamW
            optim_args.setdefault("lr", a.learning_rate)
            optim_args.setdefault("weight_decay", a.weight_decay)
            optim_args.setdefault("betas", (a.adam_beta1, a.adam_beta2))
            optim_args.setdefault("eps", a.adam_epsilon)
        dl_args = {"batch_size": a.per_device_train_batch_size * self._world_hint(), "shuffle": a.shuffle,
                   "num_workers": a.dataloader_num_workers, "drop_last": a.dataloader_drop_last,
                   "pin_memory": torch.cuda.is_available()}
        if self.data_collator is None and a.use_default_data_collator and self.tokenizer is not None:
            from transformers import DataCollatorWithPadding

            self.data_collator = DataCollatorWithPadding(self.tokenizer)
        if self.data_collator is not None:
            dl_args["collate_fn"] = self.data_collator
        ok, res, strategy = auto_accelerate(
            self.model, optim_func if self.optimizer is None else None, dataset=self.train_dataset,
            loss_func=a.loss_func, prepare_input=a.prepare_input, model_input_format=a.model_input_format,
            optim_args=optim_args, optim_param_func=a.optim_param_func, dataloader_args=dl_args,
            load_strategy=self._build_strategy(), sampler_seed=a.seed, excluded=a.excluded, included=a.included,
            distributed_sampler_cls=a.distributed_sampler_cls)
        if not ok:
            raise RuntimeError("auto_accelerate failed")
        if a.save_strategy_to_file and self._rank() == 0:
            import json

            path = a.save_strategy_to_file if os.path.isabs(a.save_strategy_to_file) else \
                os.path.join(a.output_dir, a.save_strategy_to_file)
            os.makedirs(os.path.dirname(path) or ".", exist_ok=True)
            with open(path, "w") as f:
                json.dump([[n, repr(c) if c is not None else None] for n, c in strategy.opts], f, indent=1)
        self.model = res.model
        self.optimizer = self.optimizer or res.optim
        self.train_dataloader = res.dataloader
        self.prepare_input = res.prepare_input
        self.loss_func = res.loss_func
        self.device = res.args.get("device", torch.device("cpu"))
        self.amp_dtype = res.args.get("amp_dtype")
        self.grad_scaler = res.args.get("grad_scaler")
        self.strategy = strategy
        self.is_fsdp = any(n in ("fsdp", "zero2") for n in strategy.names())

    def _world_hint(self) -> int:
        if dist.is_initialized():
            return dist.get_world_size()
        return int(os.environ.get("WORLD_SIZE", "1"))

    def create_scheduler(self, num_training_steps: int, optimizer=None):
        from transformers import get_scheduler

        if self.lr_scheduler is None:
            self.lr_scheduler = get_scheduler(self.args.atorch_lr_scheduler_type or self.args.lr_scheduler_type,
                                              optimizer=optimizer or self.optimizer,
                                              num_warmup_steps=self.args.get_warmup_steps(num_training_steps),
                                              num_training_steps=num_training_steps)
        return self.lr_scheduler

    # ---------------------------------------------------------------- steps
    def _prepare_inputs(self, inputs):
        return self.prepare_input(inputs, self.device) if self.prepare_input else inputs

    def compute_loss(self, model, inputs, return_outputs=False):
        fmt = self.args.model_input_format
        if fmt == "unpack_dict" and isinstance(inputs, dict):
            outputs = model(**inputs)
        elif fmt == "unpack_sequence" and isinstance(inputs, (list, tuple)):
            outputs = model(*inputs)
        else:
            outputs = model(inputs)
        if self.loss_func is not None:
            loss = self.loss_func(inputs, outputs)
        elif torch.is_tensor(outputs) and outputs.dim() == 0:
            loss = outputs
        elif isinstance(outputs, dict) or hasattr(outputs, "loss"):
            loss = outputs["loss"] if isinstance(outputs, dict) else outputs.loss
        else:
            loss = outputs[0]
        if isinstance(loss, (tuple, list)):
            loss = loss[0]
        return (loss, outputs) if return_outputs else loss

    def _autocast(self):
        if self.amp_dtype is None or self.is_fsdp:
            import contextlib

            return contextlib.nullcontext()
        return torch.autocast(self.device.type, dtype=self.amp_dtype)

    def training_step(self, model, inputs) -> torch.Tensor:
        model.train()
        inputs = self._prepare_inputs(inputs)
        with self._autocast():
            loss = self.compute_loss(model, inputs)
        loss = loss / self.args.gradient_accumulation_steps
        if self.grad_scaler is not None:
            self.grad_scaler.scale(loss).backward()
        else:
            loss.backward()
        return loss.detach()

    def _clip(self) -> Optional[torch.Tensor]:
        if not self.args.max_grad_norm or self.args.max_grad_norm <= 0:
            return None
        if self.grad_scaler is not None:
            self.grad_scaler.unscale_(self.optimizer)
        params = [p for p in self.model.parameters() if p.grad is not None]
        return torch.nn.utils.clip_grad_norm_(params, self.args.max_grad_norm)

    # ---------------------------------------------------------------- train
    def train(self, resume_from_checkpoint=None, **kwargs):
        args = self.args
        if resume_from_checkpoint is True:
            resume_from_checkpoint = self._latest_checkpoint()
        self._set_seed(args.seed)
        dl = self.train_dataloader
        if dl is None:
            raise ValueError("AtorchTrainer needs a train_dataset")
        ga = max(1, args.gradient_accumulation_steps)
        len_dl = len(dl) if hasattr(dl, "__len__") else None
        if args.max_steps > 0:
            max_steps = args.max_steps
            steps_per_epoch = max(1, (len_dl or max_steps * ga) // ga)
            num_epochs = math.ceil(max_steps / steps_per_epoch)
        else:
            if len_dl is None:
                raise ValueError("max_steps must be set when the dataloader has no length")
            steps_per_epoch = max(1, len_dl // ga)
            max_steps = math.ceil(args.num_train_epochs * steps_per_epoch)
            num_epochs = math.ceil(args.num_train_epochs)
        self.create_scheduler(max_steps)
        self.callback_handler.optimizer = self.optimizer
        self.callback_handler.lr_scheduler = self.lr_scheduler
        self.callback_handler.train_dataloader = dl
        self.state = TrainerState()
        self.state.max_steps = max_steps
        self.state.num_train_epochs = num_epochs
        self.state.logging_steps, self.state.eval_steps, self.state.save_steps = (
            args.logging_steps, args.eval_steps, args.save_steps)
        self.state.is_local_process_zero = self.is_local_process_zero()
        self.state.is_world_process_zero = self.is_world_process_zero()
        epochs_done, skip_batches = 0, 0
        if resume_from_checkpoint:
            self._load_checkpoint(resume_from_checkpoint)
            epochs_done = self.state.global_step // steps_per_epoch
            skip_batches = (self.state.global_step % steps_per_epoch) * ga
        tot, trainable = _count_params(self.model)
        logger.info(f"AtorchTrainer: {trainable:,}/{tot:,} trainable params, {max_steps} steps, "
                    f"strategy {self.strategy.names()}")
        self.control = self.callback_handler.on_train_begin(args, self.state, self.control)
        tr_loss = torch.zeros((), device=self.device)
        logged_loss, last_log_step = 0.0, self.state.global_step
        start = time.time()
        self.optimizer.zero_grad(set_to_none=True)
        for epoch in range(epochs_done, num_epochs):
            sampler = getattr(dl, "sampler", None)
            if hasattr(sampler, "set_epoch"):
                sampler.set_epoch(epoch)
            self.control = self.callback_handler.on_epoch_begin(args, self.state, self.control)
            for step, inputs in enumerate(dl):
                if skip_batches > 0:
                    skip_batches -= 1
                    continue
                last_micro = (step + 1) % ga == 0 or (len_dl is not None and step + 1 == len_dl)
                if step % ga == 0:
                    self.control = self.callback_handler.on_step_begin(args, self.state, self.control)
                sync = last_micro or not hasattr(self.model, "no_sync")
                ctx = self.model.no_sync() if not sync else _null()
                with ctx:
                    tr_loss += self.training_step(self.model, inputs)
                if not last_micro:
                    continue
                norm = self._clip()
                finite = norm is None or bool(torch.isfinite(norm))
                if finite or not args.skip_if_nonfinite:
                    if self.grad_scaler is not None:
                        self.grad_scaler.step(self.optimizer)
                        self.grad_scaler.update()
                    else:
                        self.optimizer.step()
                    self.lr_scheduler.step()
                else:
                    logger.warning(f"step {self.state.global_step + 1}: non-finite grad norm, skipped")
                self.optimizer.zero_grad(set_to_none=True)
                self.state.global_step += 1
                self.state.epoch = epoch + (step + 1) / max(1, len_dl or 1)
                self.control = self.callback_handler.on_step_end(args, self.state, self.control)
                if self.control.should_log:
                    cur = float(tr_loss)
                    n = max(1, self.state.global_step - last_log_step)
                    logs = {"loss": round((cur - logged_loss) / n, 6),
                            "learning_rate": self.lr_scheduler.get_last_lr()[0],
                            "grad_norm": float(norm) if norm is not None else None, "epoch": self.state.epoch}
                    logged_loss, last_log_step = cur, self.state.global_step
                    self.log(logs)
                if self.control.should_evaluate and self.eval_dataset is not None:
                    self.evaluate()
                if self.control.should_save:
                    try:
                        self._save_checkpoint()
                    except OSError as e:
                        if not args.ignore_write_errors:
                            raise
                        logger.warning(f"checkpoint write failed at step {self.state.global_step} "
                                       f"(ignore_write_errors): {e}")
                    self.control = self.callback_handler.on_save(args, self.state, self.control)
                if self.control.should_training_stop or self.state.global_step >= max_steps:
                    break
            self.control = self.callback_handler.on_epoch_end(args, self.state, self.control)
            if self.control.should_training_stop or self.state.global_step >= max_steps:
                break
        if self._checkpointer is not None and hasattr(self._checkpointer, "wait_latest_checkpoint"):
            self._checkpointer.wait_latest_checkpoint()
        if args.load_best_model_at_end and self.state.best_model_checkpoint:
            self._load_best_model()
        runtime = time.time() - start
        metrics = {"train_runtime": round(runtime, 4), "train_loss": float(tr_loss) / max(1, self.state.global_step),
                   "global_step": self.state.global_step}
        self.control = self.callback_handler.on_train_end(args, self.state, self.control)
        return TrainResult(self.state.global_step, metrics["train_loss"], metrics)

    def log(self, logs: Dict[str, float]):
        logs = {k: v for k, v in logs.items() if v is not None}
        logs["step"] = self.state.global_step
        self.state.log_history.append(logs)
        self.control = self.callback_handler.on_log(self.args, self.state, self.control, logs)

    # ---------------------------------------------------------------- eval
    def get_eval_dataloader(self, eval_dataset=None):
        ds = eval_dataset if eval_dataset is not None else self.eval_dataset
        bs = self.args.per_device_eval_batch_size
        if dist.is_initialized() and dist.get_world_size() > 1:
            # contiguous runs of whole batches per rank: the rank-ordered
            # gather is the dataset order, and padding batches are whole
            # batches the loop runs (matched collectives) but does not record
            bsm = DistributedEvalBatchSampler(len(ds), bs, dist.get_world_size(), dist.get_rank())
            return torch.utils.data.DataLoader(ds, batch_sampler=bsm, collate_fn=self.data_collator)
        return torch.utils.data.DataLoader(ds, batch_size=bs, collate_fn=self.data_collator)

    def _logits(self, out):
        if torch.is_tensor(out):
            return out
        if isinstance(out, dict) or hasattr(out, "keys"):
            for k in (self.args.logit_names or ["logits"]):
                if k in out:
                    return out[k]
            return None
        if hasattr(out, "logits"):
            return out.logits
        if isinstance(out, (tuple, list)) and len(out) > 1:
            return out[self.args.logit_index]
        return None

    @staticmethod
    def _labels(inputs):
        if isinstance(inputs, dict):
            for k in ("labels", "label", "label_ids", "targets"):
                if k in inputs and torch.is_tensor(inputs[k]):
                    return inputs[k]
        return None

    @staticmethod
    def _batch_size(inputs) -> int:
        if torch.is_tensor(inputs):
            return inputs.shape[0]
        vals = inputs.values() if isinstance(inputs, dict) else inputs if isinstance(inputs, (list, tuple)) else []
        for v in vals:
            if torch.is_tensor(v) and v.dim() > 0:
                return v.shape[0]
        return 1

    def _comm_device(self):
        return self.device if dist.is_initialized() and dist.get_backend() == "nccl" else torch.device("cpu")

    _DTYPES = (torch.float32, torch.float16, torch.bfloat16, torch.float64, torch.int64, torch.int32, torch.int16,
               torch.int8, torch.uint8, torch.bool)
    _MAX_DIMS = 8

    def _gather(self, t: Optional[torch.Tensor], counts: List[int], pad_index=-100) -> Optional[torch.Tensor]:
        """Rank-ordered concatenation over the data-parallel ranks of each
        rank's first ``counts[rank]`` rows.  COLLECTIVE: every rank calls it,
        a rank without rows with ``t=None`` -- the dtype and trailing shape
        are agreed first (max over ranks), the tensors padded with
        ``pad_index`` to a common shape for the all-gather, then trimmed.
        Returns None on every rank when no rank has a tensor."""
        world = self._world()
        if world == 1:
            return t
        dev = self._comm_device()
        nd = self._MAX_DIMS
        meta = torch.zeros(2 + nd, dtype=torch.int64, device=dev)
        if t is not None:
            if t.dim() > nd or t.dtype not in self._DTYPES:
                raise ValueError(f"cannot gather a {t.dtype} tensor of {t.dim()} dims")
            meta[0] = 1 + self._DTYPES.index(t.dtype)
            meta[1] = t.dim()
            meta[2:2 + t.dim()] = torch.tensor(list(t.shape), dtype=torch.int64)
        dist.all_reduce(meta, op=dist.ReduceOp.MAX)
        m = [int(x) for x in meta.tolist()]
        if m[0] == 0:
            return None
        dtype, ndim = self._DTYPES[m[0] - 1], m[1]
        want = [max(counts)] + m[3:2 + ndim]
        out = torch.full(want, pad_index, dtype=dtype, device=dev)
        if t is not None and t.numel():
            out[tuple(slice(0, n) for n in t.shape)] = t.to(dev, dtype)
        parts = [torch.empty_like(out) for _ in range(world)]
        dist.all_gather(parts, out)
        return torch.cat([p[:c] for p, c in zip(parts, counts)])

    def _counts(self, rows: int) -> List[int]:
        """Every rank's row count (collective)."""
        if self._world() == 1:
            return [rows]
        c = torch.zeros(self._world(), dtype=torch.int64, device=self._comm_device())
        c[self._rank()] = rows
        dist.all_reduce(c)
        return [int(x) for x in c.tolist()]

    def evaluation_loop(self, dataset, metric_key_prefix: str = "eval", want_preds: bool = False):
        """Loss, predictions and labels over the WHOLE dataset, in dataset
        order, on every rank (reference ``evaluation_loop`` /
        ``_nested_gather``, atorch_trainer.py:1857-2043).

        Memory-bounded like the reference (atorch_trainer.py:149,203-207,
        1903-1961): ``preprocess_logits_for_metrics(logits, labels)`` runs
        per batch on the device (e.g. vocab logits -> argmax ids), logits
        keep their own dtype, and with ``eval_accumulation_steps = k`` the
        device-side accumulation is gathered across the ranks and moved to
        the host every k batches -- the device holds at most k batches (x
        world while gathering) whatever the dataset length.  Without it the
        accumulation stays on the device and is gathered once at the end
        (no host sync per batch).  Gathers are collectives every rank
        enters, ranks whose share is only padding batches included."""
        dl = self.get_eval_dataloader(dataset)
        n = len(dl.dataset)
        real_batches = getattr(dl.batch_sampler, "num_real_batches", None)
        eas = self.args.eval_accumulation_steps or 0
        world = self._world()
        self.model.eval()
        losses, preds, labels = [], [], []  # device-side, since the last flush
        host = {"loss": [[] for _ in range(world)], "pred": [[] for _ in range(world)],
                "label": [[] for _ in range(world)]}
        collect = want_preds or self.compute_metrics is not None
        pre = self.preprocess_logits_for_metrics
        peak = 0

        def flush():
            nonlocal losses, preds, labels
            counts = self._counts(sum(x.numel() for x in losses))
            for key, buf in (("loss", losses), ("pred", preds), ("label", labels)):
                local = _pad_cat(buf) if buf else None
                g = self._gather(local, counts) if world > 1 else local
                if g is None:
                    continue
                g = g.cpu()
                o = 0
                for r, c in enumerate(counts):  # per rank: the final order is rank-major (dataset order)
                    if c:
                        host[key][r].append(g[o:o + c])
                    o += c
            losses, preds, labels = [], [], []

        with torch.no_grad():
            for bi, inputs in enumerate(dl):
                inputs = self._prepare_inputs(inputs)
                with self._autocast():
                    loss, out = self.compute_loss(self.model, inputs, return_outputs=True)
                if real_batches is None or bi < real_batches:  # else a padding batch (collectives matched)
                    bs = self._batch_size(inputs)
                    losses.append(loss.detach().float().reshape(1).expand(bs))
                    if collect:
                        lg = self._logits(out)
                        lb = self._labels(inputs)
                        if lg is not None and pre is not None:
                            lg = pre(lg, lb)
                        if lg is not None:
                            preds.append(lg.detach())
                        if lb is not None:
                            labels.append(lb.detach())
                    peak = max(peak, sum(t.numel() * t.element_size() for t in preds + labels))
                del out
                if eas and (bi + 1) % eas == 0:
                    flush()
        flush()
        self.model.train()
        self.eval_peak_accum_bytes = peak  # device bytes of accumulated predictions + labels at most

        def cat(key):
            parts = [t for r in range(world) for t in host[key][r]]
            if not parts:
                return None
            t = _pad_cat(parts)
            return t.float() if t.dtype in (torch.bfloat16, torch.float16) else t  # numpy has no bf16

        loss_all, preds_all, labels_all = cat("loss"), cat("pred"), cat("label")
        metrics = {f"{metric_key_prefix}_loss": float(loss_all.mean()) if loss_all is not None else float("nan")}
        if self.compute_metrics is not None and preds_all is not None:
            from transformers import EvalPrediction

            m = self.compute_metrics(EvalPrediction(predictions=preds_all.numpy(),
                                                    label_ids=labels_all.numpy() if labels_all is not None else None))
            metrics.update({k if k.startswith(metric_key_prefix + "_") else f"{metric_key_prefix}_{k}": v
                            for k, v in m.items()})
        metrics[f"{metric_key_prefix}_samples"] = n
        return EvalLoopOutput(preds_all, labels_all, metrics, n)

    def evaluate(self, eval_dataset=None, metric_key_prefix: str = "eval") -> Dict[str, float]:
        ds = eval_dataset if eval_dataset is not None else self.eval_dataset
        out = self.evaluation_loop(ds, metric_key_prefix)
        metrics = out.metrics
        self._last_eval_metrics = dict(metrics)
        self.log(dict(metrics))
        self.control = self.callback_handler.on_evaluate(self.args, self.state, self.control, metrics)
        return metrics

    def predict(self, test_dataset, metric_key_prefix: str = "test") -> "EvalLoopOutput":
        """Predictions (and labels / metrics when the dataset has labels) of
        the whole dataset, in dataset order, on every rank."""
        return self.evaluation_loop(test_dataset, metric_key_prefix, want_preds=True)

    # ---------------------------------------------------------------- best model
    def _track_best(self, ckpt_dir: str):
        """At a save: is the last evaluation the best so far?  (HF
        ``_determine_best_metric``; reference atorch_trainer.py:1304
        ``_save_checkpoint``)."""
        a = self.args
        metrics = getattr(self, "_last_eval_metrics", None)
        if not metrics or not a.metric_for_best_model:
            return
        name = a.metric_for_best_model
        if not name.startswith("eval_"):
            name = f"eval_{name}"
        if name not in metrics:
            logger.warning(f"metric_for_best_model {name} not in the evaluation metrics {sorted(metrics)}")
            return
        v = float(metrics[name])
        greater = a.greater_is_better if a.greater_is_better is not None else not name.endswith("loss")
        best = self.state.best_metric
        if best is None or (v > best if greater else v < best):
            self.state.best_metric = v
            self.state.best_model_checkpoint = ckpt_dir
            if hasattr(self.state, "best_global_step"):
                self.state.best_global_step = self.state.global_step

    def _load_best_model(self):
        """``load_best_model_at_end``: the weights of the best checkpoint
        (reference atorch_trainer.py:1197)."""
        d = self.state.best_model_checkpoint
        if not d or not os.path.isdir(d):
            logger.warning("load_best_model_at_end: no best checkpoint recorded")
            return
        if self._checkpointer is not None and hasattr(self._checkpointer, "wait_latest_checkpoint"):
            self._checkpointer.wait_latest_checkpoint()  # its async persist may still be writing
        if self.is_fsdp:
            from torch.distributed.checkpoint.state_dict import get_model_state_dict, set_model_state_dict

            import torch.distributed.checkpoint as dcp

            msd = get_model_state_dict(self.model)
            dcp.load({"model": msd}, checkpoint_id=os.path.join(d, "dcp"))
            set_model_state_dict(self.model, msd)
        else:
            path = os.path.join(d, f"rank_{self._rank()}_{STATE_FILE}")
            if not os.path.exists(path):  # replicated (DDP) flash checkpoints are persisted by rank 0 only
                path = os.path.join(d, f"rank_0_{STATE_FILE}")
            sd = torch.load(path, map_location="cpu", weights_only=True)
            if "model_states" in sd and "model" not in sd:  # flash-checkpoint archive layout
                sd = sd["model_states"]
            self.model.load_state_dict(sd["model"])
        logger.info(f"loaded the best model ({self.args.metric_for_best_model}={self.state.best_metric}) from {d}")

    # ---------------------------------------------------------------- checkpoint
    def _set_seed(self, seed: int):
        random.seed(seed)
        np.random.seed(seed)
        torch.manual_seed(seed)

    def _rng_state(self):
        st = {"python": random.getstate(), "numpy": np.random.get_state(), "cpu": torch.get_rng_state()}
        if torch.cuda.is_available():
            st["cuda"] = torch.cuda.get_rng_state()
        return st

    def _set_rng_state(self, st):
        random.setstate(st["python"])
        np.random.set_state(st["numpy"])
        torch.set_rng_state(st["cpu"])
        if "cuda" in st and torch.cuda.is_available():
            torch.cuda.set_rng_state(st["cuda"])

    def _ckpt_dir(self, step: int) -> str:
        return os.path.join(self.args.output_dir, f"{PREFIX_CHECKPOINT_DIR}-{step}")

    def _state_dict(self) -> Dict[str, Any]:
        return {"model": self.model.state_dict(), "optimizer": self.optimizer.state_dict(),
                "lr_scheduler": self.lr_scheduler.state_dict() if self.lr_scheduler else None,
                "grad_scaler": self.grad_scaler.state_dict() if self.grad_scaler else None,
                "global_step": self.state.global_step}

    def _get_checkpointer(self):
        if self._checkpointer is None:
            from ..flash_checkpoint.ddp import DdpCheckpointer

            self._checkpointer = DdpCheckpointer(self.args.output_dir)
        return self._checkpointer

    def _save_checkpoint(self):
        step = self.state.global_step
        out = self._ckpt_dir(step)
        os.makedirs(out, exist_ok=True)
        sd = self._state_dict()
        path = os.path.join(out, f"rank_{self._rank()}_{STATE_FILE}")
        if self.args.flash_checkpoint and not self.is_fsdp:
            from ..flash_checkpoint.checkpointer import StorageType

            ck = self._get_checkpointer()
            ck.save_checkpoint(step, sd, path=path, storage_type=StorageType.DISK)
            if not self.args.async_save:
                ck.wait_latest_checkpoint()
        elif self.is_fsdp:
            from torch.distributed.checkpoint.state_dict import get_state_dict

            import torch.distributed.checkpoint as dcp

            msd, osd = get_state_dict(self.model, self.optimizer)
            dcp.save({"model": msd, "optimizer": osd}, checkpoint_id=os.path.join(out, "dcp"))
            extra = {k: v for k, v in sd.items() if k not in ("model", "optimizer")}
            torch.save(extra, path)
        else:
            torch.save(sd, path)
        torch.save(self._rng_state(), os.path.join(out, f"rng_state_{self._rank()}.pth"))
        self._track_best(out)
        if self.is_world_process_zero():
            self.state.save_to_json(os.path.join(out, TRAINER_STATE_NAME))
            with open(os.path.join(self.args.output_dir, "latest_checkpoint.txt"), "w") as f:
                f.write(os.path.basename(out))
            self._rotate_checkpoints()

    def _sorted_checkpoints(self) -> List[str]:
        out = []
        for d in os.listdir(self.args.output_dir):
            m = re.match(rf"{PREFIX_CHECKPOINT_DIR}-(\d+)$", d)
            if m and os.path.isdir(os.path.join(self.args.output_dir, d)):
                out.append((int(m.group(1)), os.path.join(self.args.output_dir, d)))
        return [p for _, p in sorted(out)]

    def _rotate_checkpoints(self):
        limit = self.args.save_total_limit
        if not limit or limit <= 0:
            return
        cks = self._sorted_checkpoints()
        best = self.state.best_model_checkpoint
        if best in cks:
            # the best checkpoint is kept on top of the limit (HF semantics)
            cks.remove(best)
            limit = max(1, limit - 1) if self.args.load_best_model_at_end else limit
        for old in cks[:max(0, len(cks) - limit)]:
            logger.info(f"deleting old checkpoint {old} (save_total_limit={limit})")
            shutil.rmtree(old, ignore_errors=True)

    def _latest_checkpoint(self) -> Optional[str]:
        cks = self._sorted_checkpoints()
        return cks[-1] if cks else None

    def _load_checkpoint(self, ckpt_dir: str):
        path = os.path.join(ckpt_dir, f"rank_{self._rank()}_{STATE_FILE}")
        if self.is_fsdp:
            from torch.distributed.checkpoint.state_dict import get_state_dict, set_state_dict

            import torch.distributed.checkpoint as dcp

            msd, osd = get_state_dict(self.model, self.optimizer)
            sd = {"model": msd, "optimizer": osd}
            dcp.load(sd, checkpoint_id=os.path.join(ckpt_dir, "dcp"))
            set_state_dict(self.model, self.optimizer, model_state_dict=sd["model"], optim_state_dict=sd["optimizer"])
            extra = torch.load(path, map_location="cpu", weights_only=True)
        else:
            sd = None
            if self.args.flash_checkpoint:
                ck = self._get_checkpointer()
                got = ck.load_checkpoint(resume_path=path)
                sd = got if got else None
            if sd is None:
                sd = torch.load(path, map_location="cpu", weights_only=True)
            self.model.load_state_dict(sd["model"])
            self.optimizer.load_state_dict(sd["optimizer"])
            extra = sd
        if extra.get("lr_scheduler") is not None and self.lr_scheduler is not None:
            self.lr_scheduler.load_state_dict(extra["lr_scheduler"])
        if extra.get("grad_scaler") is not None and self.grad_scaler is not None:
            self.grad_scaler.load_state_dict(extra["grad_scaler"])
        st_path = os.path.join(ckpt_dir, TRAINER_STATE_NAME)
        if os.path.exists(st_path):
            self.state = TrainerState.load_from_json(st_path)
        else:
            self.state.global_step = int(extra.get("global_step", 0))
        rng = os.path.join(ckpt_dir, f"rng_state_{self._rank()}.pth")
        if os.path.exists(rng):
            self._set_rng_state(safe_torch_load(rng))  # numpy RNG tuple: allow-listed unpickler
        logger.info(f"resumed from {ckpt_dir} at step {self.state.global_step}")

    def save_model(self, output_dir: Optional[str] = None):
        """Final weights as safetensors (rank 0, gathered for FSDP)."""
        from safetensors.torch import save_file

        output_dir = output_dir or self.args.output_dir
        os.makedirs(output_dir, exist_ok=True)
        if self.is_fsdp:
            from torch.distributed.checkpoint.state_dict import StateDictOptions, get_model_state_dict

            sd = get_model_state_dict(self.model, options=StateDictOptions(full_state_dict=True, cpu_offload=True))
        else:
            m = self.model.module if hasattr(self.model, "module") else self.model
            sd = m.state_dict()
        if self.is_world_process_zero():
            seen, out = {}, {}
            for k, v in sd.items():
                v = v.detach().cpu().contiguous()
                key = v.data_ptr()
                out[k] = v.clone() if key in seen else v  # tied weights: safetensors forbids shared storage
                seen[key] = k
            save_file(out, os.path.join(output_dir, "model.safetensors"))
            with open(os.path.join(output_dir, "atorch_strategy.json"), "w") as f:
                json.dump([str(n) for n in self.strategy.names()], f)

    def close(self):
        if self._checkpointer is not None:
            self._checkpointer.close()
            self._checkpointer = None


class EvalLoopOutput(NamedTuple):
    """HF ``EvalLoopOutput`` / ``PredictionOutput``."""

    predictions: Optional[torch.Tensor]
    label_ids: Optional[torch.Tensor]
    metrics: Dict[str, Any]
    num_samples: int


class DistributedEvalBatchSampler(torch.utils.data.Sampler):
    """Evaluation batches for data-parallel ranks: the dataset's sequential
    batches (``[0, bs), [bs, 2 bs), ...``, only the last one partial) are
    split into contiguous runs, rank r taking batches ``[r * pb, (r + 1) *
    pb)``; ranks with fewer real batches run whole padding batches so every
    rank runs ``pb`` batches.  Padding never shares a batch with real samples,
    so per-batch mean losses weight exactly like one process, and the
    rank-ordered gather of the real rows is the dataset order."""

    def __init__(self, n: int, batch_size: int, num_replicas: int, rank: int):
        bs = max(1, batch_size)
        batches = [list(range(i, min(i + bs, n))) for i in range(0, n, bs)]
        pb = -(-len(batches) // num_replicas) if batches else 0
        mine = batches[rank * pb: (rank + 1) * pb]
        self.num_real_batches = len(mine)
        self.num_real = sum(len(b) for b in mine)
        self.batches = mine + [batches[0]] * (pb - len(mine))

    def __iter__(self):
        return iter(self.batches)

    def __len__(self):
        return len(self.batches)


def _pad_cat(ts: List[torch.Tensor], pad_index=-100) -> torch.Tensor:
    """Concatenate along dim 0, padding the other dims to the largest
    (variable sequence lengths across batches)."""
    if len({tuple(t.shape[1:]) for t in ts}) <= 1:
        return torch.cat(ts)
    shape = [max(t.shape[d] for t in ts) for d in range(1, ts[0].dim())]
    out = ts[0].new_full([sum(t.shape[0] for t in ts)] + shape, pad_index)
    o = 0
    for t in ts:
        out[(slice(o, o + t.shape[0]),) + tuple(slice(0, n) for n in t.shape[1:])] = t
        o += t.shape[0]
    return out


class _null:
    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False
