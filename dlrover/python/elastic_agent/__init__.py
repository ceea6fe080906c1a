"""Compatibility import path (reference: dlrover/python/elastic_agent).

Thin re-export onto the MI355X-native implementation in ``dlrover_wuqiong_amd.elastic_agent``;
existing DLRover / ATorch user code imports unchanged.
"""

