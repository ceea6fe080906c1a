"""Compatibility import path (reference: atorch/atorch/distributed/run.py:313,366 (python -m atorch.distributed.run)).

Thin re-export onto the MI355X-native implementation in ``dlrover_wuqiong_amd.trainer.run``;
existing DLRover / ATorch user code imports unchanged.
"""

import sys

from dlrover_wuqiong_amd.trainer.run import main  # noqa: F401

if __name__ == "__main__":
    sys.exit(main())
