"""Compatibility import path (reference: dlrover/trainer/torch/elastic).

Thin re-export onto the MI355X-native implementation in ``dlrover_wuqiong_amd.trainer.elastic``;
existing DLRover / ATorch user code imports unchanged.
"""

