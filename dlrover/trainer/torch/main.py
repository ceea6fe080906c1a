"""Compatibility import path (reference: dlrover/trainer/torch/main.py (dlrover-run console script)).

Thin re-export onto the MI355X-native implementation in ``dlrover_wuqiong_amd.trainer.run``;
existing DLRover / ATorch user code imports unchanged.
"""

import sys

from dlrover_wuqiong_amd.trainer.run import main, parse_args, run  # noqa: F401

if __name__ == "__main__":
    sys.exit(main())
