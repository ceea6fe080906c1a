"""Compatibility import path (reference: dlrover/python/master/main.py:60-70).

Thin re-export onto the MI355X-native implementation in ``dlrover_wuqiong_amd.master.master``;
existing DLRover / ATorch user code imports unchanged.
"""

import sys

from dlrover_wuqiong_amd.master.master import main  # noqa: F401

if __name__ == "__main__":
    sys.exit(main())
