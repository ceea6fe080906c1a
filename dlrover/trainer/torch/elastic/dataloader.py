"""Compatibility import path (reference: dlrover/trainer/torch/elastic/dataloader.py:26-147).

Thin re-export onto the MI355X-native implementation in ``dlrover_wuqiong_amd.trainer.elastic``;
existing DLRover / ATorch user code imports unchanged.
"""

from dlrover_wuqiong_amd.trainer.elastic import ElasticDataLoader  # noqa: F401
