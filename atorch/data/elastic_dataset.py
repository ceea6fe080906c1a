"""Compatibility import path (reference: atorch/atorch/data/elastic_dataset.py).

Thin re-export onto the MI355X-native implementation; existing ATorch user code imports unchanged.
"""

from dlrover_wuqiong_amd.atorch.data.elastic_dataset import ElasticDataset, SimpleElasticDataset  # noqa: F401
