"""Tuned GEMM solution tables for the library GEMMs (hipBLASLt / rocBLAS).

``scripts/tune_gemms.py`` times every hipBLASLt and rocBLAS solution for
each GEMM shape a model's training step issues (PyTorch TunableOp, rotating
inputs for cold-cache timings) and stores the fastest per shape in
``configs/tunableop/<model>_gfx950.csv``.  :func:`enable` loads such a table
read-only: shapes in it use the recorded solution, others the library
default; nothing is tuned at run time.  The table's validator lines pin the
PyTorch / ROCm / hipBLASLt / rocBLAS versions -- on any other stack PyTorch
rejects it and the default heuristics stay in use.

``DWAMD_GEMM_TUNING=0`` disables it.
"""

import os
from typing import Optional

from ..common.log import logger

_DIR = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "configs", "tunableop")


def table_path(model: str) -> str:
    return os.path.join(_DIR, f"{model}_gfx950.csv")


def enable(model: str, path: Optional[str] = None) -> bool:
    """Use the tuned table of ``model`` if one exists.  Returns True when
    loaded.  Call before the first GEMM of the process."""
    import torch

    if os.environ.get("DWAMD_GEMM_TUNING", "1") != "1" or not torch.cuda.is_available():
        return False
    path = path or table_path(model)
    if not os.path.exists(path):
        return False
    import torch.cuda.tunable as tun

    tun.enable(True)
    tun.tuning_enable(False)
    tun.record_untuned_enable(False)
    tun.set_filename(path, False)
    ok = bool(tun.read_file(path))
    if not ok:
        tun.enable(False)
        logger.warning(f"GEMM tuning table {path} rejected (different software stack?): library defaults")
    return ok
