"""ATorch data utilities (parity: ``atorch/atorch/data``)."""

from .elastic_dataset import ElasticDataset, SimpleElasticDataset  # noqa: F401
from .preloader import GpuPreLoader  # noqa: F401
from .shm_dataloader import ShmDataLoader, coworker_produce, create_shm_dataloader  # noqa: F401
from .shm_ring import BROADCAST, SHARED, ShmBatchRing  # noqa: F401
from .unordered_dataloader import UnorderedDataLoader  # noqa: F401

ShmDataloader = ShmDataLoader  # reference spelling
