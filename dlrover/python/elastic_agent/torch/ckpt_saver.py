"""Compatibility import path (reference: dlrover/python/elastic_agent/torch/ckpt_saver.py).

Thin re-export onto the MI355X-native implementation in ``dlrover_wuqiong_amd.elastic_agent.ckpt_saver``;
existing DLRover / ATorch user code imports unchanged.
"""

from dlrover_wuqiong_amd.elastic_agent.ckpt_saver import (AsyncCheckpointSaver, CommonDirCheckpointSaver,  # noqa: F401
                                                          DdpCheckpointSaver, DeepSpeedCheckpointSaver,
                                                          FsdpDcpSaver, MegatronCheckpointSaver,
                                                          TempDirCheckpointSaver)
