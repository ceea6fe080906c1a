"""Compatibility import path (reference: atorch/atorch/rl/data/data_utils.py).

Thin re-export onto the MI355X-native implementation in ``dlrover_wuqiong_amd.atorch.rl``;
existing ATorch user code imports unchanged.
"""

from dlrover_wuqiong_amd.atorch.rl.rl_config import PromptDataset, create_dataset, read_prompts  # noqa: F401
