"""Compatibility import path (reference: dlrover/python/elastic_agent/torch/training.py).

Thin re-export onto the MI355X-native implementation in ``dlrover_wuqiong_amd.elastic_agent.agent``;
existing DLRover / ATorch user code imports unchanged.
"""

from dlrover_wuqiong_amd.elastic_agent.agent import (ElasticLaunchConfig, ElasticTrainingAgent,  # noqa: F401
                                                     MasterRendezvousHandler, launch_agent)
