"""Diagnosis data records exchanged between agents and the master.

Parity: reference ``dlrover/python/common/diagnosis.py:18-76`` (``CudaLog``,
``TrainingLog``, ``ChipMetrics`` -- placeholders there).  Here they carry
content: ``GpuRuntimeLog`` (HIP/RCCL/driver error lines found in worker
logs; ``CudaLog`` is kept as the reference-compatible alias),
``TrainingLog`` (tail of the worker logs) and ``ChipMetrics`` (per-GPU
utilisation / memory / temperature / power from the amdgpu sysfs).
"""

import json
import time
from dataclasses import asdict, dataclass, field
from typing import Dict, List


class DiagnosisDataType:
    CUDALOG = "cuda_log"
    GPULOG = "cuda_log"  # same wire name as the reference
    TRAININGLOG = "training_log"
    CHIPMETRICES = "chip_metrics"


@dataclass
class DiagnosisData:
    timestamp: float = 0.0

    def __post_init__(self):
        if not self.timestamp:
            self.timestamp = time.time()

    def get_timestamp(self) -> float:
        return self.timestamp

    def get_type(self) -> str:
        raise NotImplementedError

    def to_json(self) -> str:
        return json.dumps(asdict(self))

    @classmethod
    def from_json(cls, s: str):
        return cls(**json.loads(s))


@dataclass
class GpuRuntimeLog(DiagnosisData):
    """Error lines matched in the worker logs (HIP / RCCL / KFD)."""

    errors: List[str] = field(default_factory=list)
    local_rank: int = -1

    def get_type(self) -> str:
        return DiagnosisDataType.CUDALOG


CudaLog = GpuRuntimeLog


@dataclass
class TrainingLog(DiagnosisData):
    logs: List[str] = field(default_factory=list)

    def get_type(self) -> str:
        return DiagnosisDataType.TRAININGLOG


@dataclass
class ChipMetrics(DiagnosisData):
    """Per-GPU metrics keyed by GPU index (str for JSON)."""

    gpus: Dict[str, Dict[str, float]] = field(default_factory=dict)

    def get_type(self) -> str:
        return DiagnosisDataType.CHIPMETRICES


DATA_CLASSES = {"GpuRuntimeLog": GpuRuntimeLog, "CudaLog": GpuRuntimeLog, "TrainingLog": TrainingLog,
                "ChipMetrics": ChipMetrics}
