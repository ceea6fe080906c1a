"""Datasets whose sample indices come from the job master's dynamic data
sharding service, so nodes never read duplicates in an epoch and a
restarted/added node picks up the remaining shards.

Parity: ATorch ``atorch/data/elastic_dataset.py`` (``ElasticDataset.read_sample``,
``report_batch_done``, ``SimpleElasticDataset``).
"""

from abc import ABCMeta, abstractmethod
from typing import Callable

from torch.utils.data import Dataset


class ElasticDataset(Dataset, metaclass=ABCMeta):
    def __init__(self, name: str, dataset_size: int, batch_size: int, epochs: int, shuffle: bool = False,
                 num_minibatches_per_shard: int = 2, master_client=None):
        from ...elastic_agent.sharding_client import IndexShardingClient

        self._shard_client = IndexShardingClient(dataset_name=name, batch_size=batch_size, num_epochs=epochs,
                                                 dataset_size=dataset_size, shuffle=shuffle,
                                                 num_minibatches_per_shard=num_minibatches_per_shard,
                                                 storage_type="text", master_client=master_client)

    def __len__(self):
        return self._shard_client.get_total_sample_num()

    def __getitem__(self, _):
        index = self._shard_client.fetch_sample_index()
        if index is None:
            raise IndexError("dataset exhausted")
        return self.read_sample(index)

    def report_batch_done(self, batch_size=None):
        self._shard_client.report_batch_done(batch_size)

    def state_dict(self):
        return {"shard_checkpoint": self._shard_client.get_shard_checkpoint()}

    def load_state_dict(self, state):
        if state and state.get("shard_checkpoint"):
            self._shard_client.restore_shard_from_checkpoint(state["shard_checkpoint"])

    @abstractmethod
    def read_sample(self, index):
        """Read one sample by its global index."""


class SimpleElasticDataset(ElasticDataset):
    def __init__(self, name: str, data_process_fn: Callable, dataset_size: int, batch_size: int, epochs: int,
                 shuffle: bool = False, num_minibatches_per_shard: int = 2, master_client=None):
        self.data_process_fn = data_process_fn
        super().__init__(name, dataset_size, batch_size, epochs, shuffle, num_minibatches_per_shard,
                         master_client)

    def read_sample(self, index):
        return self.data_process_fn(index)
