"""Compatibility import path (reference: atorch/atorch/rl/main.py).

Thin re-export onto the MI355X-native implementation in ``dlrover_wuqiong_amd.atorch.rl``;
existing ATorch user code imports unchanged.
"""

from dlrover_wuqiong_amd.atorch.rl.main import main, parse_args, rl_train  # noqa: F401

if __name__ == "__main__":
    main()
