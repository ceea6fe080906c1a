"""Parallelism-config tuner: bridges the master's suggestions into the
JSON file that ``ElasticDataLoader`` / ``auto_accelerate`` re-read.

Every ``interval`` seconds: report the local config (dataloader batch size,
optimizer lr ...) to the master, fetch the master's suggestion, and rewrite
the file (bumping ``version`` so readers notice).

Parity: reference ``dlrover/python/elastic_agent/config/paral_config_tuner.py:30-101``.
"""

import json
import os
import threading
from typing import Optional

from ..common import comm
from ..common.constants import ConfigPath
from ..common.log import logger
from .master_client import MasterClient


class ParalConfigTuner:
    _instance = None

    def __init__(self, master_client: Optional[MasterClient] = None, config_path: str = "",
                 interval: float = 30.0):
        self._mc = master_client or MasterClient.singleton_instance()
        self.config_path = config_path or os.getenv(ConfigPath.ENV_PARAL_CONFIG, ConfigPath.PARAL_CONFIG)
        self.config_dir = os.path.dirname(self.config_path)
        self.interval = interval
        self._stop = threading.Event()
        self._thread: Optional[threading.Thread] = None
        self._create_paral_config_file()

    @classmethod
    def singleton_instance(cls, *args, **kwargs) -> "ParalConfigTuner":
        if cls._instance is None:
            cls._instance = cls(*args, **kwargs)
        return cls._instance

    def start(self):
        if self._thread is not None:
            return
        self._thread = threading.Thread(target=self._periodically_update_paral_config, daemon=True,
                                        name="dwamd-config-tuner")
        self._thread.start()
        logger.info(f"parallelism config tuner started ({self.config_path})")

    def stop(self):
        self._stop.set()

    def _create_paral_config_file(self):
        os.makedirs(self.config_dir or ".", exist_ok=True)
        if not os.path.exists(self.config_path):
            self._write(comm.ParallelConfig())

    def _write(self, config: comm.ParallelConfig):
        d = {"dataloader": vars(config.dataloader) if config.dataloader else {},
             "optimizer": vars(config.optimizer) if config.optimizer else {},
             "restart": bool(getattr(config, "restart", False))}
        tmp = self.config_path + ".tmp"
        with open(tmp, "w") as f:
            json.dump(d, f)
        os.replace(tmp, self.config_path)

    def _read_paral_config(self) -> Optional[comm.ParallelConfig]:
        try:
            with open(self.config_path) as f:
                data = json.load(f)
        except (FileNotFoundError, json.JSONDecodeError) as e:
            logger.warning(f"cannot read {self.config_path}: {e}")
            return None
        return comm.ParallelConfig(dataloader=comm.DataLoaderConfig(**data.get("dataloader", {})),
                                   optimizer=comm.OptimizerConfig(**data.get("optimizer", {})))

    def update_once(self):
        local = self._read_paral_config()
        if local is not None:
            self._mc.report_paral_config(local)
        cfg = self._mc.get_paral_config()
        if cfg is not None and cfg.dataloader is not None and (cfg.dataloader.version or 0) > 0:
            if local is None or cfg.dataloader.version != local.dataloader.version:
                self._write(cfg)
                logger.info(f"applied parallelism config version {cfg.dataloader.version}")

    def _periodically_update_paral_config(self):
        while not self._stop.wait(self.interval):
            try:
                self.update_once()
            except Exception as e:
                logger.debug(f"config tuner: {e}")
