"""Rank / world-size helpers read from the launcher environment.

Parity: reference ``dlrover/python/common/env_utils.py:17-74``.
"""

import os

from .constants import NodeEnv


def _int_env(name: str, default: int) -> int:
    v = os.getenv(name)
    if v is None or v == "":
        return default
    try:
        return int(v)
    except ValueError:
        return default


def get_node_rank() -> int:
    """Rank of this node (agent) in the job."""
    return _int_env(NodeEnv.NODE_RANK, _int_env("GROUP_RANK", 0))


def get_local_rank() -> int:
    return _int_env("LOCAL_RANK", 0)


def get_rank() -> int:
    return _int_env("RANK", 0)


def get_world_size() -> int:
    return _int_env("WORLD_SIZE", 1)


def get_local_world_size() -> int:
    return _int_env("LOCAL_WORLD_SIZE", 1)


def get_group_rank() -> int:
    return _int_env("GROUP_RANK", get_node_rank())


def get_group_world_size() -> int:
    return _int_env("GROUP_WORLD_SIZE", get_node_num())


def get_torch_restart_count() -> int:
    return _int_env("TORCHELASTIC_RESTART_COUNT", 0)


def get_node_num() -> int:
    return _int_env(NodeEnv.NODE_NUM, 1)


def get_node_id() -> int:
    return _int_env(NodeEnv.NODE_ID, get_node_rank())


def get_job_name() -> str:
    return os.getenv(NodeEnv.JOB_NAME, os.getenv(NodeEnv.TORCHELASTIC_RUN_ID, "local"))


def get_run_id() -> str:
    return os.getenv(NodeEnv.TORCHELASTIC_RUN_ID, "")


def is_under_agent() -> bool:
    return os.getenv("ROLE_NAME", "") == "dlrover-trainer"
