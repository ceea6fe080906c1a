"""Compatibility import path (reference: atorch/atorch/rl/replay_buffer/replay_buffer.py).

Thin re-export onto the MI355X-native implementation in ``dlrover_wuqiong_amd.atorch.rl``;
existing ATorch user code imports unchanged.
"""

from dlrover_wuqiong_amd.atorch.rl.replay_buffer import SampleReplayBuffer as ReplayBuffer  # noqa: F401
