"""Compatibility import path (reference: dlrover/trainer/torch/elastic_run.py:125-391).

Thin re-export onto the MI355X-native implementation in ``dlrover_wuqiong_amd.trainer.run``;
existing DLRover / ATorch user code imports unchanged.
"""

import sys

from dlrover_wuqiong_amd.trainer.run import build_config, launch_local_master, main, parse_args, run  # noqa: F401

if __name__ == "__main__":
    sys.exit(main())
