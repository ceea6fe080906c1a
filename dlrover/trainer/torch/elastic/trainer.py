"""Compatibility import path (reference: dlrover/trainer/torch/elastic/trainer.py:181-336).

Thin re-export onto the MI355X-native implementation in ``dlrover_wuqiong_amd.trainer.elastic``;
existing DLRover / ATorch user code imports unchanged.
"""

from dlrover_wuqiong_amd.trainer.elastic import ElasticTrainer  # noqa: F401
