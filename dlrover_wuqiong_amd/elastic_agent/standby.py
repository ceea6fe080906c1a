"""Warm standby workers: pre-started processes that become the next workers.

Restarting a worker after a fault normally costs a fresh ``python`` +
``import torch`` + HIP init + model build + kernel warm-up + pinning the
checkpoint shm before the first useful step.  The agent therefore keeps one
*standby* process per local rank ready.  Two modes:

``import`` (default, safe for any script)
    The standby imports torch and this package, initialises the HIP runtime
    on its local rank's GPU and keeps this rank's part of the node's
    checkpoint shm pinned (``DWAMD_STANDBY_GPU_INIT=0``: touch no GPU, for
    scripts that choose their visible devices in-process), and blocks on
    stdin.  On (re)start the agent sends one JSON line -- worker
    environment, argv, entrypoint, log file -- and the standby turns into
    the worker in place (``runpy``, ``__main__`` semantics).  The script
    still builds its model and restores: the reference's restart semantics,
    minus interpreter start, imports, HIP init and the pinning of the restore
    source.  Like a deep standby it owns the live worker's HBM checkpoint
    staging buffers (HBM tier, when they fit; ``DWAMD_HBM_TIER=0``: off), so
    a worker killed while its last snapshot was still flushing to shm
    restores that step D2D instead of losing a checkpoint interval.

``deep`` (opt-in: ``dwamd-run --standby-mode deep``; the script must call
:func:`standby_point`)
    The standby runs the training script *immediately* with a provisional
    environment (``LOCAL_RANK`` / ``LOCAL_WORLD_SIZE`` known, no ``RANK`` /
    ``WORLD_SIZE`` / ``MASTER_*``).  The script does everything that does not
    need the world -- HIP init, model + optimizer allocation on its GPU,
    kernel warm-up -- and then calls :func:`standby_point`, which pins this
    rank's part of the node's checkpoint shm (so the restore is a plain DMA),
    reports readiness to the agent and blocks.  At activation it applies the
    real worker environment and returns; the script continues with
    ``init_process_group``, restores from shm and trains.  A restart is then
    rendezvous + RCCL init + H2D restore.  On MI355X the standby's copy of the
    model fits next to the live worker (288 GB HBM per GPU).

No ``exec`` anywhere: a process that has initialised the GPU is never
replaced; it simply continues as the worker.

The reference (torchelastic-based agent, ``training.py:580-645,704``) always
cold-starts workers; this is an MI355X-deployment goodput optimisation
measured by ``bench.py``.
"""

import importlib
import json
import os
import runpy
import sys
import time
from typing import Optional

STANDBY_ENV = "DWAMD_STANDBY"
SPEC_ENV = "DWAMD_STANDBY_SPEC"
READY_PREFIX = "standby_ready."

_activated: Optional[dict] = None
_STREAM = None  # import standby: the stream its HBM reservation belongs to (the worker's current stream)


def is_standby() -> bool:
    """True in a deep standby that has not been activated yet."""
    return os.environ.get(STANDBY_ENV, "0") == "1" and _activated is None


def _preload():
    mods = os.environ.get("DWAMD_STANDBY_PRELOAD", "torch,torch.distributed,dlrover_wuqiong_amd.flash_checkpoint.ddp")
    for m in filter(None, (x.strip() for x in mods.split(","))):
        try:
            importlib.import_module(m)
        except Exception as e:  # a missing optional module must not kill the standby
            print(f"[standby] preload {m} failed: {e}", file=sys.stderr)
    try:
        # the first torch.optim.Optimizer of a process imports torch._dynamo
        # (~900 modules, ~1.1 s): pay it here, not inside the restart
        import torch

        torch.optim.SGD([torch.zeros(1, requires_grad=True)], lr=0.1)
    except Exception as e:
        print(f"[standby] optimizer warm-up failed: {e}", file=sys.stderr)


def _redirect(log_path: str):
    if not log_path:
        return
    os.makedirs(os.path.dirname(log_path) or ".", exist_ok=True)
    fd = os.open(log_path, os.O_WRONLY | os.O_CREAT | os.O_TRUNC, 0o644)
    sys.stdout.flush()
    sys.stderr.flush()
    os.dup2(fd, 1)
    os.dup2(fd, 2)
    os.close(fd)


def _apply(cmd: dict):
    _redirect(cmd.get("log", ""))
    os.environ.clear()
    os.environ.update(cmd["env"])
    if cmd.get("cwd"):
        os.chdir(cmd["cwd"])


PINNED_PREFIX = "standby_pinned."
WARM_PREFIX = "standby_warm."  # the warm profile was replayed (value: bytes reserved)


def _prepin_checkpoint_shm() -> float:
    """Map + hipHostRegister this local rank's part of the node's flash
    checkpoint segments (kept for the checkpoint engine to adopt).  Returns
    seconds spent; idempotent (re-pins only a re-created segment)."""
    try:
        from ..flash_checkpoint.prewarm import prepin_local_checkpoint_shm

        return prepin_local_checkpoint_shm()
    except Exception as e:  # never fatal: the restore pins on demand
        print(f"[standby] shm pre-pin skipped: {e}", file=sys.stderr)
        return 0.0


def _pinned_bytes() -> int:
    try:
        from ..flash_checkpoint.prewarm import prepinned_bytes

        return prepinned_bytes()
    except Exception:
        return 0


STAGING_PREFIX = "standby_staging."  # staging buffers held for the worker (value: bytes, tier on/off)
RESERVED_PREFIX = "standby_reserved."  # restart-path HBM reserved (value: bytes held for the worker)


def _publish_hbm_staging(ctl: str, lr: str):
    """Hold the worker's checkpoint staging buffers in this standby.  HBM
    tier on: publish them to the live worker (they outlive it, the standby
    restores D2D).  Tier off: keep them private -- the worker this standby
    becomes snapshots into them, so no save after a restart allocates VRAM.
    Also reserves the replicated restore's all-gather temporary (N > 1)."""
    try:
        from ..flash_checkpoint import hbm_tier
        from ..flash_checkpoint.prewarm import local_slice_bytes, restore_temp_bytes

        n = local_slice_bytes()
        if n <= 0:
            return
        tier = os.environ.get("DWAMD_HBM_TIER", "1") == "1"
        ok = (hbm_tier.publish_standby_buffers(ctl, int(lr), n) if tier else
              hbm_tier.reserve_private_staging(n))
        tmp = hbm_tier.reserve_restore_temp(restore_temp_bytes())
        if ok and ctl and not os.path.exists(os.path.join(ctl, STAGING_PREFIX + lr)):
            _mark(ctl, STAGING_PREFIX, lr, f"{2 * n} {int(tier)} {tmp}\n")
    except Exception as e:  # never fatal: the restore falls back to shm
        print(f"[standby] HBM staging not held: {e}", file=sys.stderr)


def _mark(ctl: str, prefix: str, lr: str, text: str):
    if not ctl:
        return
    path = os.path.join(ctl, prefix + lr)
    with open(path + ".tmp", "w") as f:
        f.write(text)
    os.replace(path + ".tmp", path)


def standby_point(prepin_shm: bool = True, repin_interval: float = 0.25) -> Optional[dict]:
    """Call once in the training script after world-independent set-up.

    Not a standby: returns ``None`` immediately.  Deep standby: signals
    readiness and blocks until the agent activates this process (returns
    ``{"activated_at": t, "waited_s": s, "prepin_s": p}``) or discards it
    (the process exits 0 without returning).  While parked it keeps this
    rank's part of the node's checkpoint shm pinned (the segment may appear,
    or be re-created at a new size, only after the standby parked).
    """
    global _activated
    if not is_standby():
        return None
    import select

    ctl = os.environ.get("DWAMD_AGENT_CTL_DIR", "")
    lr = os.environ.get("LOCAL_RANK", "0")
    pin_s = _prepin_checkpoint_shm() if prepin_shm else 0.0
    if prepin_shm:
        _publish_hbm_staging(ctl, lr)
    _mark(ctl, READY_PREFIX, lr, f"{os.getpid()} {time.time()}\n")
    pinned_marked = False
    t0 = time.time()
    buf = b""
    fd = sys.stdin.fileno()
    cmd = None
    rsv = _Reservation(ctl, lr, deep=True) if prepin_shm else None
    while cmd is None:
        if not pinned_marked and prepin_shm and _pinned_bytes() > 0:
            _mark(ctl, PINNED_PREFIX, lr, f"{_pinned_bytes()}\n")
            pinned_marked = True
        if rsv is not None:
            rsv.tick()
        r, _, _ = select.select([fd], [], [], repin_interval)
        if r:
            chunk = os.read(fd, 1 << 20)
            if not chunk:
                sys.stdout.flush()
                sys.stderr.flush()
                os._exit(0)  # discarded by the agent (stdin closed)
            buf += chunk
            buf, cmd = _control_lines(buf, ctl, lr)
        elif prepin_shm:
            pin_s += _prepin_checkpoint_shm()
            _publish_hbm_staging(ctl, lr)
    _apply(cmd)
    from . import pg_preform

    pg_preform.arm(bool(cmd.get("adopt_pg")))
    _activated = {"activated_at": time.time(), "waited_s": time.time() - t0, "prepin_s": pin_s,
                  "pinned_bytes": _pinned_bytes(), "pg_preformed": pg_preform.preformed()}
    return dict(_activated)


def _control_lines(buf: bytes, ctl: str, lr: str):
    """Consume complete JSON lines from the agent: ``preform`` requests are
    served in place (pg_preform.py); the first other line is the activation
    command.  Returns (rest of the buffer, activation command or None)."""
    from . import pg_preform

    while b"\n" in buf:
        line, buf = buf.split(b"\n", 1)
        if not line.strip():
            continue
        obj = json.loads(line.decode())
        if pg_preform.handle_line(obj, ctl, lr):
            continue
        return buf, obj
    return buf, None


def reserved_stream():
    """The stream an import standby made current (its reservation's stream),
    else None."""
    return _STREAM


def activation_info() -> Optional[dict]:
    return dict(_activated) if _activated else None


def _run_entry(entry: str, args, module: bool):
    sys.argv = [entry] + list(args)
    if module:
        runpy.run_module(entry, run_name="__main__", alter_sys=True)
    else:
        sys.path.insert(0, os.path.dirname(os.path.abspath(entry)))
        runpy.run_path(entry, run_name="__main__")


def _gpu_init(lr: str) -> bool:
    """HIP runtime + a context on this rank's device (import mode)."""
    try:
        import torch

        if not torch.cuda.is_available():
            return False
        torch.cuda.set_device(int(lr) % max(1, torch.cuda.device_count()))
        # PyTorch's caching allocator reuses a freed block only for the
        # stream it was allocated on: everything this standby reserves for the
        # worker it becomes is allocated on ONE non-blocking stream, which
        # stays the current stream when the script runs (a script that keeps
        # the current stream -- or asks dlrover_wuqiong_amd.trainer.elastic.
        # training_stream() -- allocates from the reservation; one that
        # switches to a stream of its own allocates from the driver)
        global _STREAM
        if os.environ.get("DWAMD_STANDBY_STREAM", "1") == "1":
            _STREAM = torch.cuda.Stream()
            torch.cuda.set_stream(_STREAM)
        # ... and the checkpoint flush stream right after it: HIP maps the
        # streams of one priority round-robin onto GPU_MAX_HW_QUEUES (4)
        # hardware queues, and a flush stream created after RCCL's streams
        # landed on the compute stream's queue (each step after a save waited
        # for the 0.4 s flush; profiles/r6/bench_1gpu_import_queue_sharing.json)
        from ..flash_checkpoint.copier import precreate_flush_stream

        if os.environ.get("DWAMD_STANDBY_FLUSH_STREAM", "1") == "1":
            precreate_flush_stream(torch.device("cuda", torch.cuda.current_device()))
        x = torch.ones(64, 64, device="cuda", dtype=torch.bfloat16)
        (x @ x).float().sum().item()  # BLAS handle + a first kernel launch
        from .._native import kernels

        kernels(required=False)  # this package's HIP kernel library (code objects registered)
        for m in os.environ.get("DWAMD_STANDBY_PRELOAD_GPU", "dlrover_wuqiong_amd.models.gpt2,"
                                "dlrover_wuqiong_amd.models.llama,dlrover_wuqiong_amd.optimizers.fused,"
                                "dlrover_wuqiong_amd.parallel.ddp,dlrover_wuqiong_amd.parallel.flat").split(","):
            if m.strip():
                try:
                    importlib.import_module(m.strip())
                except Exception as e:
                    print(f"[standby] preload {m} failed: {e}", file=sys.stderr)
        torch.cuda.synchronize()
        return True
    except Exception as e:  # never fatal: the worker initialises on its own
        print(f"[standby] GPU pre-init skipped: {e}", file=sys.stderr)
        return False


def _reserve_state_memory(reserved: int = 0, prof: Optional[dict] = None, held: int = 0) -> int:
    """Fill PyTorch's caching allocator with about the HBM the worker will
    take -- its recorded peak footprint (warm profile: model + optimizer +
    activations), else the checkpoint payload size once a save made it known
    -- and leave it cached: the driver's allocation of fresh VRAM (it clears
    every new buffer) is then paid while waiting, not inside the restart
    (~1.9 s for the 19 GB of GPT2-1.5B Adam state alone).  ``reserved``:
    bytes already held (only the increment is allocated); ``held``: bytes
    of the worker's footprint this process already holds otherwise (a deep
    standby's built model + optimizer).  Bounded by the free HBM;
    DWAMD_STANDBY_RESERVE=0 disables it.  Returns bytes reserved (-1:
    skipped for good)."""
    if os.environ.get("DWAMD_STANDBY_RESERVE", "1") != "1":
        return -1
    try:
        import torch

        from ..flash_checkpoint.prewarm import local_state_bytes
        from .warm_profile import reserve_bytes

        want = reserve_bytes(prof, local_state_bytes(), float(os.environ.get("DWAMD_STANDBY_RESERVE_FACTOR", "1.25")))
        want -= held
        if want <= reserved:
            return reserved
        free, _total = torch.cuda.mem_get_info()
        n = min(want - reserved, int(free * 0.8) - (8 << 30))
        if n <= (1 << 30):
            return reserved or -1  # no room next to the live worker
        t = torch.empty(n, dtype=torch.uint8, device="cuda")
        del t  # stays in the allocator's cache for the worker this process becomes
        return reserved + n
    except Exception as e:  # never fatal
        print(f"[standby] HBM reserve skipped: {e}", file=sys.stderr)
        return reserved or -1


class _Reservation:
    """Everything a restart would otherwise allocate from the driver, held
    by the standby while it waits (``DWAMD_STANDBY_RESERVE=0``: off):

    * the worker's peak footprint in the caching allocator (import: the
      whole peak; deep: the peak minus the model + optimizer it already
      built -- the first steps' activations);
    * 128 MiB of small-block pool (descriptor tables, scalars, batches);
    * checkpoint staging + the restore all-gather temporary
      (:func:`_publish_hbm_staging`).

    The counter the bench reports (``device_allocs_after_restart``) is the
    allocator's device allocations from activation to the 4th save after
    the restart; with these held it is 0.  Released under HBM pressure."""

    def __init__(self, ctl: str, lr: str, deep: bool):
        self.ctl, self.lr, self.deep = ctl, lr, deep
        self.reserved = 0
        self.prof = None
        self.small = False
        self.marked = False
        self.held = 0

    def tick(self, replay_profile: bool = False):
        if os.environ.get("DWAMD_STANDBY_RESERVE", "1") != "1":
            return
        if not self.small:
            try:
                from ..flash_checkpoint.hbm_tier import reserve_small_pool

                reserve_small_pool()
            except Exception as e:  # never fatal
                print(f"[standby] small-pool reserve skipped: {e}", file=sys.stderr)
            self.small = True
            if self.deep:
                import torch

                self.held = int(torch.cuda.memory_allocated())  # the built model + optimizer
        if self.prof is None:
            if replay_profile:
                self.prof = _apply_warm_profile(self.ctl, self.lr)
            else:
                from . import warm_profile

                self.prof = warm_profile.load(self.ctl, self.lr) if self.ctl else None
            if self.prof is not None:
                if self.reserved >= 0:
                    self.reserved = _reserve_state_memory(self.reserved, self.prof, self.held)
                _mark(self.ctl, WARM_PREFIX, self.lr, f"{self.reserved}\n")
                self._mark_reserved()
        if self.reserved == 0 and not self.deep:
            self.reserved = _reserve_state_memory()
        elif self.reserved > 0:
            self.reserved = _release_under_pressure(self.reserved)

    def _mark_reserved(self):
        if not self.marked:
            _mark(self.ctl, RESERVED_PREFIX, self.lr, f"{max(0, self.reserved)}\n")
            self.marked = True


def _apply_warm_profile(ctl: str, lr: str) -> Optional[dict]:
    """Replay the live worker's warm profile (its GEMMs) once it exists."""
    from . import warm_profile

    prof = warm_profile.load(ctl, lr) if ctl else None
    if prof is None:
        return None
    try:
        warm_profile.preload_kernel_library()
        r = warm_profile.replay(prof)
        print(f"[standby] warm profile replayed: {r['gemms']} GEMMs, {r.get('ops', 0)} other ops "
              f"({r['failed']} failed) in {r['sec']} s", file=sys.stderr)
    except Exception as e:  # never fatal
        print(f"[standby] warm profile replay failed: {e}", file=sys.stderr)
    return prof


def _release_under_pressure(reserved: int) -> int:
    """The reservation lives next to the LIVE worker on the same GPU: when
    the device's free HBM drops under ``DWAMD_STANDBY_RELEASE_GB`` (default
    max(16 GiB, 6 % of the card)) -- the worker's eval / activation peak /
    its staging buffers want it -- hand the cached blocks back to the driver
    and stop reserving.  Returns the new reservation state (-1 = released
    for good)."""
    if reserved <= 0:
        return reserved
    try:
        import torch

        free, total = torch.cuda.mem_get_info()
        floor = float(os.environ.get("DWAMD_STANDBY_RELEASE_GB", "0")) * (1 << 30) or max(16 << 30, 0.06 * total)
        if free < floor:
            torch.cuda.empty_cache()
            print(f"[standby] released {reserved / 2**30:.1f} GiB reserved HBM (device free "
                  f"{free / 2**30:.1f} GiB < {floor / 2**30:.1f} GiB)", file=sys.stderr)
            return -1
    except Exception as e:  # never fatal
        print(f"[standby] release check failed: {e}", file=sys.stderr)
    return reserved


def _wait_command(pin: bool, ctl: str, lr: str, interval: float = 0.25) -> Optional[dict]:
    """Block until the agent's activation line arrives on stdin (served
    ``preform`` requests on the way); meanwhile keep this rank's checkpoint
    shm pinned (segments appear, or are re-created at a new size, while the
    standby waits).  None = discarded."""
    import select

    buf = b""
    fd = sys.stdin.fileno()
    pinned_marked = False
    rsv = _Reservation(ctl, lr, deep=False)
    cmd = None
    while cmd is None:
        if pin:
            _prepin_checkpoint_shm()
            _publish_hbm_staging(ctl, lr)
            if not pinned_marked and _pinned_bytes() > 0:
                _mark(ctl, PINNED_PREFIX, lr, f"{_pinned_bytes()}\n")
                pinned_marked = True
            rsv.tick(replay_profile=True)
        r, _, _ = select.select([fd], [], [], interval)
        if r:
            chunk = os.read(fd, 1 << 20)
            if not chunk:
                return None
            buf += chunk
            buf, cmd = _control_lines(buf, ctl, lr)
    return cmd


def main():
    spec = os.environ.get(SPEC_ENV, "")
    if spec:
        # deep standby: run the script now; it blocks in standby_point()
        s = json.loads(spec)
        _redirect(s.get("log", ""))
        if s.get("cwd"):
            os.chdir(s["cwd"])
        os.environ.pop(SPEC_ENV, None)
        _run_entry(s["entry"], s.get("args", []), s.get("module", False))
        if _activated is None:
            # the script finished without ever reaching standby_point(): it is
            # not standby-aware; report and exit non-zero so the agent cold-starts
            print("[standby] script returned before standby_point(); not a deep-standby script",
                  file=sys.stderr)
            return 3
        return 0
    _preload()
    ctl = os.environ.get("DWAMD_AGENT_CTL_DIR", "")
    lr = os.environ.get("DWAMD_STANDBY_LOCAL_RANK", "0")
    gpu = os.environ.get("DWAMD_STANDBY_GPU_INIT", "1") == "1" and _gpu_init(lr)
    if gpu:
        os.environ.setdefault("LOCAL_RANK", lr)  # the shm pre-pin pins this rank's ranges
    # import mode: torch + this package are imported; tell the agent (and
    # anyone waiting on the control dir) this standby can take over now
    _mark(ctl, READY_PREFIX, lr, f"{os.getpid()} {time.time()}\n")
    cmd = _wait_command(gpu, ctl, lr)
    if cmd is None:
        return 0  # agent discarded the standby
    _apply(cmd)
    from . import pg_preform

    pg_preform.arm(bool(cmd.get("adopt_pg")))
    _run_entry(cmd["entry"], cmd.get("args", []), cmd.get("module", False))
    return 0


if __name__ == "__main__":
    sys.exit(main())
