"""Compatibility import path (reference: atorch/atorch/utils/sparse.py).

Thin re-export onto the MI355X-native implementation in ``dlrover_wuqiong_amd.atorch.utils.sparse``;
existing ATorch user code imports unchanged.
"""

from dlrover_wuqiong_amd.atorch.utils.sparse import all_reduce_sparse  # noqa: F401
