"""Pre-formed process groups: RCCL world formation off the recovery path.

After a fault the replacement workers normally pay rendezvous + RCCL
bootstrap (unique-id exchange, topology discovery, per-peer xGMI buffer
set-up and IPC handle exchange) before their first collective -- on an
8 x MI355X node that is the largest single item of a restart once the
restore itself is a DMA from host shm or HBM.  The reference always pays
it: its agent restarts workers through torchelastic and every worker calls
``init_process_group`` cold (``dlrover/python/elastic_agent/torch/
training.py:411-545,704``).

Here the node's standbys (one per local rank, ``standby.py``) form their
communicator while they are parked, long before anything fails:

1. once every local standby of a generation is parked, the agent sends
   each one a ``{"preform": {...}}`` line on its stdin: the address of a
   TCPStore the agent hosts, a per-generation key prefix, the backend and
   the group size (the node's local world);
2. the standby runs ``init_process_group`` over that store with
   ``rank = LOCAL_RANK`` (eager RCCL init on its GPU, ``device_id``) and one
   all-reduce, then writes ``standby_pg.<local rank>`` into the agent's
   control dir;
3. at the restart the agent activates the standbys with ``adopt_pg``:
   true only when the new world is exactly this node's local ranks (the
   single-node job: ``WORLD_SIZE == LOCAL_WORLD_SIZE``, ``RANK ==
   LOCAL_RANK``) and every standby of the set reported a formed group.
   The script's own ``init_process_group`` call then returns at once with
   the pre-formed group as the default group (``adopted() is True``);
   with ``adopt_pg`` false -- membership changed, a standby missing -- the
   pre-formed group is destroyed first and the script's call forms the new
   world cold.

A requested backend that differs from the pre-formed one (e.g. a script
that asks for gloo where the standby formed RCCL) also falls back.
Collectives get a timeout (``DWAMD_COLLECTIVE_TIMEOUT_S``, default 600 s)
and the RCCL watchdog tears the process down when one expires
(``TORCH_NCCL_ASYNC_ERROR_HANDLING``), so a rank stuck on a hung peer
exits and the agent restarts the group instead of the job hanging.
"""

import datetime
import os
import sys
import time
from typing import Optional

PG_MARK_PREFIX = "standby_pg."

_state: dict = {}  # backend, rank, world, sec, prefix (the pre-formed group, if any)
_adopted: Optional[dict] = None
_orig_init = None


def collective_timeout() -> datetime.timedelta:
    return datetime.timedelta(seconds=float(os.environ.get("DWAMD_COLLECTIVE_TIMEOUT_S", "600")))


def _log(msg: str):
    print(f"[pg-preform] {msg}", file=sys.stderr, flush=True)


def auto_backend() -> str:
    """RCCL when this process already owns a GPU context, else gloo."""
    try:
        import torch

        if torch.cuda.is_available() and torch.cuda.is_initialized():
            return "nccl"
    except Exception:
        pass
    return "gloo"


def preform(store_addr: str, prefix: str, rank: int, world: int, backend: str = "auto",
            device=None, timeout: float = 120.0) -> bool:
    """Form the standby set's process group (the default group of this
    process).  Returns True when formed; never raises (the restart then
    forms the world cold)."""
    import torch
    import torch.distributed as dist

    if dist.is_initialized():
        return bool(_state)
    backend = auto_backend() if backend in ("", "auto", None) else backend
    t0 = time.time()
    try:
        host, port = store_addr.rsplit(":", 1)
        store = dist.TCPStore(host, int(port), is_master=False, timeout=datetime.timedelta(seconds=timeout))
        kw = {}
        if backend == "nccl":
            kw["device_id"] = torch.device("cuda", torch.cuda.current_device()) if device is None else device
        dist.init_process_group(backend, store=dist.PrefixStore(prefix, store), rank=rank, world_size=world,
                                timeout=collective_timeout(), **kw)
        dev = kw.get("device_id", torch.device("cpu"))
        t = torch.ones(1, device=dev)
        dist.all_reduce(t)  # the communicator exists and every peer answered
        if dev.type == "cuda":
            torch.cuda.synchronize(dev)
        ok = float(t.item()) == float(world)
        # the pre-form limit guarded the rendezvous only: later store waits
        # (subgroup unique ids after an adoption) get the collective timeout
        store.set_timeout(collective_timeout())
    except Exception as e:
        _log(f"pre-forming a {backend} group of {world} failed: {e}")
        _destroy()
        return False
    if not ok:
        _log("pre-formed group answered a wrong all-reduce: dropped")
        _destroy()
        return False
    _state.clear()
    _state.update(backend=backend, rank=rank, world=world, sec=round(time.time() - t0, 4), prefix=prefix)
    _log(f"{backend} group of {world} pre-formed as rank {rank} in {_state['sec']} s")
    return True


def preformed() -> Optional[dict]:
    return dict(_state) if _state else None


def adopted() -> Optional[dict]:
    """Set when the script's init_process_group adopted the pre-formed group."""
    return dict(_adopted) if _adopted else None


def _destroy():
    _state.clear()
    try:
        import torch.distributed as dist

        if dist.is_initialized():
            dist.destroy_process_group()
    except Exception as e:
        _log(f"destroying the pre-formed group failed: {e}")


def _compatible(backend, world_size: int, rank: int) -> bool:
    if not _state:
        return False
    if backend not in (None, ""):
        b = str(backend).lower()
        want = _state["backend"]
        # "nccl", or a device map such as "cpu:gloo,cuda:nccl" naming it
        if b != want and not (":" in b and want in b.replace(",", ":").split(":")):
            return False
    env_world = int(os.environ.get("WORLD_SIZE", "-1"))
    env_rank = int(os.environ.get("RANK", "-1"))
    world_size = env_world if world_size in (None, -1) else world_size
    rank = env_rank if rank in (None, -1) else rank
    return world_size == _state["world"] and rank == _state["rank"]


_rebound: list = []  # (namespace dict, name) rebound to the wrapper at arm()
# big third-party trees that never call init_process_group themselves (the
# scan is on the restart path; torch's own entry points are patched above)
_SKIP_MODULES = frozenset(("torch", "numpy", "scipy", "pandas", "pyarrow", "sympy", "encodings", "importlib"))


_alias_sites: Optional[list] = None  # (namespace dict, name) found while parked


def _find_aliases(orig) -> list:
    out = []
    for mname, mod in list(sys.modules.items()):
        if mod is None or mname.split(".", 1)[0] in _SKIP_MODULES:
            continue
        d = getattr(mod, "__dict__", None)
        if not isinstance(d, dict) or d is globals():  # (this module keeps the original in _orig_init)
            continue
        try:
            out.extend((d, k) for k, v in d.items() if v is orig)
        except RuntimeError:  # the dict changed under us (another thread importing)
            continue
    return out


def _rebind_aliases(orig, wrapper) -> int:
    """Point every module-global name that IS ``orig`` at ``wrapper``: a
    script that did ``from torch.distributed import init_process_group``
    before a deep standby parked holds the original function in its own
    globals (``__main__``, the runpy module of the script, or any of its
    modules); patching the torch attributes alone would leave it calling
    the original, which then finds the pre-formed default group and raises
    "trying to initialize the default process group twice"."""
    global _alias_sites
    # a deep standby scanned while parked (the script is blocked in
    # standby_point, so nothing new binds the name): the restart only rebinds
    sites = _alias_sites if _alias_sites is not None else _find_aliases(orig)
    _alias_sites = None
    n = 0
    for d, k in sites:
        if d.get(k) is orig:
            d[k] = wrapper
            _rebound.append((d, k))
            n += 1
    return n


def arm(adopt: bool):
    """Called once at activation.  ``adopt`` (the agent's decision): keep the
    pre-formed group for the script's ``init_process_group``; else drop it.

    The first ``init_process_group`` call after this -- through
    ``torch.distributed``, ``distributed_c10d`` or any module-global alias of
    the function -- adopts the group when the request matches it (backend,
    world, rank), else destroys it and forms the world cold; either way the
    patch and every rebound alias are undone by that call."""
    global _orig_init
    if not _state:
        return
    if not adopt:
        t0 = time.time()
        _destroy()
        _log(f"not adopted (world changed or a standby is missing): destroyed in {time.time() - t0:.3f} s")
        return
    import torch.distributed as dist
    import torch.distributed.distributed_c10d as c10d

    if _orig_init is not None:
        return
    _orig_init = orig = c10d.init_process_group

    def init_process_group(backend=None, init_method=None, timeout=None, world_size=-1, rank=-1, store=None,
                           group_name="", pg_options=None, device_id=None, **kw):
        global _adopted
        _restore_init()
        if dist.is_initialized() and _state and _compatible(backend, world_size, rank):
            _adopted = dict(_state, adopted_at=time.time())
            _set_store_timeout(timeout)
            _log(f"adopted the pre-formed {_state['backend']} group (rank {_state['rank']} of {_state['world']})")
            return None
        if _state:
            _log(f"requested backend={backend!r} world={world_size} rank={rank} does not match the pre-formed "
                 f"{_state}: forming the world cold")
            _destroy()
        return orig(backend=backend, init_method=init_method, timeout=timeout, world_size=world_size, rank=rank,
                    store=store, group_name=group_name, pg_options=pg_options, device_id=device_id, **kw)

    c10d.init_process_group = init_process_group
    dist.init_process_group = init_process_group
    _rebound.clear()
    _rebind_aliases(orig, init_process_group)


def disarm():
    """Undo :func:`arm`'s patch without using it (the script never called
    ``init_process_group``); the pre-formed group stays the default group."""
    _restore_init()


def _set_store_timeout(timeout=None):
    """The adopted group keeps the standby's store client: give it the
    script's (or the collective) timeout instead of the pre-form limit, so
    store waits of lazily created subgroups time out like a cold world's."""
    try:
        import torch.distributed.distributed_c10d as c10d

        t = timeout if timeout is not None else collective_timeout()
        c10d._get_default_store().set_timeout(t)
    except Exception as e:  # never fatal
        _log(f"store timeout not updated: {e}")


def _restore_init():
    global _orig_init
    if _orig_init is None:
        return
    import torch.distributed as dist
    import torch.distributed.distributed_c10d as c10d

    wrapper = c10d.init_process_group
    c10d.init_process_group = _orig_init
    dist.init_process_group = _orig_init
    for d, k in _rebound:
        if d.get(k) is wrapper:
            d[k] = _orig_init
    _rebound.clear()
    _orig_init = None


def handle_line(obj: dict, ctl: str, lr: str) -> bool:
    """A ``{"preform": {...}}`` control line from the agent (see module doc).
    Returns True when it was one (the caller keeps waiting for activation)."""
    spec = obj.get("preform") if isinstance(obj, dict) else None
    if spec is None:
        return False
    global _alias_sites
    ok = preform(spec["store"], spec["prefix"], int(lr), int(spec["world"]), spec.get("backend", "auto"),
                 timeout=float(spec.get("timeout", 120.0)))
    if ok:
        import torch.distributed.distributed_c10d as c10d

        _alias_sites = _find_aliases(c10d.init_process_group)  # off the restart path
    if ok and ctl:
        path = os.path.join(ctl, PG_MARK_PREFIX + lr)
        with open(path + ".tmp", "w") as f:
            f.write(f"{spec['prefix']} {_state['backend']} {_state['sec']}\n")
        os.replace(path + ".tmp", path)
    return True


def init_process_group(backend: Optional[str] = None, **kw):
    """``torch.distributed.init_process_group`` with this framework's
    collective timeout (RCCL watchdog tears a stuck rank down) unless the
    caller passes one; adopts a pre-formed group like the patched call."""
    import torch.distributed as dist

    kw.setdefault("timeout", collective_timeout())
    return dist.init_process_group(backend, **kw)
