"""DataLoader that yields batches in completion order: one slow sample (a
huge image, a remote read) no longer stalls the batches that other workers
already finished.

Parity: ATorch ``atorch/data/unordered_dataloader.py`` (a custom
``_MultiProcessingDataLoaderIter``); PyTorch now exposes the same behaviour
as ``DataLoader(in_order=False)``, which this builds on.
"""

from torch.utils.data import DataLoader


class UnorderedDataLoader(DataLoader):
    def __init__(self, *args, **kwargs):
        kwargs["in_order"] = False
        super().__init__(*args, **kwargs)
