"""Model-parallel process groups (TP / CP(SP) / EP / DP / PP).

Rank layout (innermost first): ``tp -> cp -> dp -> pp``; expert parallel
groups are carved out of ``dp x cp`` (EP ranks are consecutive data-parallel
ranks).  TP innermost keeps tensor-parallel collectives (the most frequent,
latency-bound all-reduce / all-gather per layer) on consecutive local GPUs --
on an MI355X node every GPU pair has a direct xGMI link, so a TP group of
up to 8 stays inside one node's fully connected xGMI mesh; DP / PP cross
nodes.

Parity: ATorch ``atorch/distributed/distributed.py`` (``parallel_group``,
``create_parallel_group``, ``parallel_rank``/``parallel_group_size``) and
Megatron ``mpu`` getters used by the reference's Megatron flash checkpoint
(``megatron_engine.py:46-60``).  All groups use the default backend (RCCL on
GPU, gloo on CPU); a gloo twin of the data-parallel group is created for
CPU-side control collectives.
"""

from dataclasses import dataclass, field
from typing import Dict, List, Optional

import torch.distributed as dist


@dataclass
class _State:
    tp: int = 1
    cp: int = 1
    ep: int = 1
    dp: int = 1
    pp: int = 1
    groups: Dict[str, object] = field(default_factory=dict)
    ranks: Dict[str, List[int]] = field(default_factory=dict)
    initialized: bool = False


_STATE = _State()


def _new_group(ranks: List[int], backend: Optional[str] = None):
    return dist.new_group(ranks=ranks, backend=backend)


def initialize_model_parallel(tensor_model_parallel_size: int = 1, pipeline_model_parallel_size: int = 1,
                              context_parallel_size: int = 1, expert_model_parallel_size: int = 1,
                              backend: Optional[str] = None):
    """Create every parallel group (collective: all ranks must call)."""
    world = dist.get_world_size()
    rank = dist.get_rank()
    tp, pp, cp, ep = (tensor_model_parallel_size, pipeline_model_parallel_size, context_parallel_size,
                      expert_model_parallel_size)
    if world % (tp * pp * cp) != 0:
        raise ValueError(f"world {world} not divisible by tp*pp*cp={tp * pp * cp}")
    dp = world // (tp * pp * cp)
    if (dp * cp) % ep != 0:
        raise ValueError(f"expert parallel size {ep} must divide dp*cp={dp * cp}")
    st = _State(tp=tp, cp=cp, ep=ep, dp=dp, pp=pp)

    def coord(r):
        t = r % tp
        c = (r // tp) % cp
        d = (r // (tp * cp)) % dp
        p = r // (tp * cp * dp)
        return t, c, d, p

    def rank_of(t, c, d, p):
        return t + tp * (c + cp * (d + dp * p))

    def build(name, members_of):
        # every rank creates every group in the same order (new_group is collective)
        seen = set()
        for r in range(world):
            members = tuple(members_of(*coord(r)))
            if members in seen:
                continue
            seen.add(members)
            g = _new_group(list(members), backend)
            if rank in members:
                st.groups[name] = g
                st.ranks[name] = list(members)

    build("tp", lambda t, c, d, p: [rank_of(x, c, d, p) for x in range(tp)])
    build("cp", lambda t, c, d, p: [rank_of(t, x, d, p) for x in range(cp)])
    build("dp", lambda t, c, d, p: [rank_of(t, c, x, p) for x in range(dp)])
    build("dp_cp", lambda t, c, d, p: [rank_of(t, xc, xd, p) for xd in range(dp) for xc in range(cp)])
    build("pp", lambda t, c, d, p: [rank_of(t, c, d, x) for x in range(pp)])
    build("mp", lambda t, c, d, p: [rank_of(xt, c, d, xp) for xp in range(pp) for xt in range(tp)])
    # first + last pipeline stage: tied input embedding / LM head gradients
    build("embd", lambda t, c, d, p: sorted({rank_of(t, c, d, 0), rank_of(t, c, d, pp - 1)}))

    def ep_members(t, c, d, p):
        flat = c + cp * d  # position inside dp_cp
        base = flat // ep * ep
        out = []
        for f in range(base, base + ep):
            out.append(rank_of(t, f % cp, f // cp, p))
        return out

    build("ep", ep_members)

    def edp_members(t, c, d, p):
        flat = c + cp * d
        off = flat % ep
        return [rank_of(t, f % cp, f // cp, p) for f in range(off, dp * cp, ep)]

    build("edp", edp_members)
    st.initialized = True
    global _STATE
    _STATE = st
    return st


def model_parallel_is_initialized() -> bool:
    return _STATE.initialized


def destroy_model_parallel():
    global _STATE
    _STATE = _State()


def _group(name):
    if not _STATE.initialized:
        return None
    return _STATE.groups.get(name)


def _rank_in(name) -> int:
    if not _STATE.initialized:
        return 0
    return _STATE.ranks[name].index(dist.get_rank())


def _size(name, attr) -> int:
    if not _STATE.initialized:
        return 1
    return len(_STATE.ranks[name])


def get_tensor_model_parallel_group():
    return _group("tp")


def get_pipeline_model_parallel_group():
    return _group("pp")


def get_data_parallel_group(with_context_parallel: bool = False):
    return _group("dp_cp" if with_context_parallel else "dp")


def get_context_parallel_group():
    return _group("cp")


def get_expert_model_parallel_group():
    return _group("ep")


def get_expert_data_parallel_group():
    return _group("edp")


def get_model_parallel_group():
    return _group("mp")


def get_embedding_group():
    return _group("embd")


def get_tensor_model_parallel_rank() -> int:
    return _rank_in("tp")


def get_pipeline_model_parallel_rank() -> int:
    return _rank_in("pp")


def get_data_parallel_rank(with_context_parallel: bool = False) -> int:
    return _rank_in("dp_cp" if with_context_parallel else "dp")


def get_context_parallel_rank() -> int:
    return _rank_in("cp")


def get_expert_model_parallel_rank() -> int:
    return _rank_in("ep")


def get_tensor_model_parallel_world_size() -> int:
    return _size("tp", "tp")


def get_pipeline_model_parallel_world_size() -> int:
    return _size("pp", "pp")


def get_data_parallel_world_size(with_context_parallel: bool = False) -> int:
    return _size("dp_cp" if with_context_parallel else "dp", "dp")


def get_context_parallel_world_size() -> int:
    return _size("cp", "cp")


def get_expert_model_parallel_world_size() -> int:
    return _size("ep", "ep")


def group_ranks(name: str) -> List[int]:
    return list(_STATE.ranks.get(name, []))


def is_pipeline_first_stage() -> bool:
    return get_pipeline_model_parallel_rank() == 0


def is_pipeline_last_stage() -> bool:
    return get_pipeline_model_parallel_rank() == get_pipeline_model_parallel_world_size() - 1
