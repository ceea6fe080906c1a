"""Compatibility import path (reference: dlrover/trainer/torch/elastic/sampler.py:25-158).

Thin re-export onto the MI355X-native implementation in ``dlrover_wuqiong_amd.trainer.elastic``;
existing DLRover / ATorch user code imports unchanged.
"""

from dlrover_wuqiong_amd.trainer.elastic import ElasticDistributedSampler  # noqa: F401
