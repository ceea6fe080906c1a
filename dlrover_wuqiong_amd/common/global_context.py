"""Master-side tunables (overridable through environment variables).

Parity: reference ``dlrover/python/common/global_context.py`` (``ConfigKeys``,
``DefaultValues``, ``Context``).  The reference can also pull these from its
Brain optimisation service; here ``DWAMD_CTX_<KEY>`` environment variables
(upper-cased ``ConfigKeys`` value) override the defaults.
"""

import os
import threading


class ConfigKeys:
    TRAIN_SPEED_RECORD_NUM = "train_speed_record_num"
    SECONDS_TO_START_AUTOSCALE_WORKER = "seconds_to_start_autoscale_worker"
    STEP_TO_ADJUST_WORKER = "step_to_adjust_worker"
    OPTIMIZE_WORKER_CPU_THRESHOLD = "optimize_worker_cpu_threshold"
    SECONDS_FOR_STABLE_WORKER_COUNT = "seconds_for_stable_worker_count"
    SECONDS_INTERVAL_TO_OPTIMIZE = "seconds_interval_to_optimize"
    FACTOR_TO_CUT_PENDING_CPU = "factor_to_cut_pending_cpu"
    FACTOR_TO_CUT_PENDING_MEM = "factor_to_cut_pending_mem"
    SECONDS_TO_WAIT_PENDING_POD = "seconds_to_wait_pending_pod"
    SECONDS_HUGE_TRAINING_THRESHOLD = "seconds_huge_training_threshold"
    GLOBAL_STEP_COUNT_TO_AUTO_WORKER = "global_step_count_to_auto_worker"
    SECONDS_TO_CHANGE_PS = "seconds_to_change_ps"
    SECONDS_TO_WAIT_FAILED_PS = "seconds_to_wait_failed_ps"
    HANG_CPU_USAGE_RATE = "hang_cpu_usage_rate"
    SECONDS_HANG_DETECTION = "seconds_hang_detection"


class DefaultValues:
    TRAIN_SPEED_RECORD_NUM = 50
    SEC_TO_START_AUTOSCALE_WORKER = 90
    STEP_TO_ADJUST_WORKER = 200
    OPTIMIZED_WORKER_CPU_THRESHOLD = 20
    SEC_FOR_STABLE_WORKER_COUNT = 60
    SEC_INTERVAL_TO_OPTIMIZE = 300
    FACTOR_TO_CUT_PENDING_CPU = 2
    FACTOR_TO_CUT_PENDING_MEM = 2
    SEC_TO_WAIT_PENDING_POD = 900
    SEC_HUGE_TRAINING_THRESHOLD = 1800
    STEP_SAMPLE_COUNT_TO_AUTO_WORKER = 5
    SEC_TO_CHANGE_PS = 3600
    SEC_TO_WAIT_FAILED_PS = 600
    HANG_CPU_USAGE_RATE = 0.05
    SEC_HANG_DETECTION = 1800


def _env(key: str, default):
    v = os.getenv("DWAMD_CTX_" + key.upper())
    if v is None:
        return default
    return type(default)(v) if not isinstance(default, bool) else v.lower() in ("1", "true", "yes")


class Context:
    _instance = None
    _lock = threading.Lock()

    def __init__(self):
        self.train_speed_record_num = _env(ConfigKeys.TRAIN_SPEED_RECORD_NUM, DefaultValues.TRAIN_SPEED_RECORD_NUM)
        self.seconds_to_autoscale_worker = _env(ConfigKeys.SECONDS_TO_START_AUTOSCALE_WORKER,
                                                DefaultValues.SEC_TO_START_AUTOSCALE_WORKER)
        self.step_to_adjust_worker = _env(ConfigKeys.STEP_TO_ADJUST_WORKER, DefaultValues.STEP_TO_ADJUST_WORKER)
        self.optimize_worker_cpu_threshold = _env(ConfigKeys.OPTIMIZE_WORKER_CPU_THRESHOLD,
                                                  DefaultValues.OPTIMIZED_WORKER_CPU_THRESHOLD)
        self.seconds_for_stable_worker_count = _env(ConfigKeys.SECONDS_FOR_STABLE_WORKER_COUNT,
                                                    DefaultValues.SEC_FOR_STABLE_WORKER_COUNT)
        self.seconds_interval_to_optimize = _env(ConfigKeys.SECONDS_INTERVAL_TO_OPTIMIZE,
                                                 DefaultValues.SEC_INTERVAL_TO_OPTIMIZE)
        self.factor_to_cut_pending_cpu = _env(ConfigKeys.FACTOR_TO_CUT_PENDING_CPU,
                                              DefaultValues.FACTOR_TO_CUT_PENDING_CPU)
        self.factor_to_cut_pending_mem = _env(ConfigKeys.FACTOR_TO_CUT_PENDING_MEM,
                                              DefaultValues.FACTOR_TO_CUT_PENDING_MEM)
        self.seconds_to_wait_pending_pod = _env(ConfigKeys.SECONDS_TO_WAIT_PENDING_POD,
                                                DefaultValues.SEC_TO_WAIT_PENDING_POD)
        self.seconds_huge_training_threshold = _env(ConfigKeys.SECONDS_HUGE_TRAINING_THRESHOLD,
                                                    DefaultValues.SEC_HUGE_TRAINING_THRESHOLD)
        self.sample_count_to_adjust_worker = _env(ConfigKeys.GLOBAL_STEP_COUNT_TO_AUTO_WORKER,
                                                  DefaultValues.STEP_SAMPLE_COUNT_TO_AUTO_WORKER)
        self.hang_cpu_usage_percentage = _env(ConfigKeys.HANG_CPU_USAGE_RATE, DefaultValues.HANG_CPU_USAGE_RATE)
        self.seconds_interval_to_change_ps = _env(ConfigKeys.SECONDS_TO_CHANGE_PS, DefaultValues.SEC_TO_CHANGE_PS)
        self.seconds_to_wait_failed_ps = _env(ConfigKeys.SECONDS_TO_WAIT_FAILED_PS,
                                              DefaultValues.SEC_TO_WAIT_FAILED_PS)
        self.seconds_hang_detection = _env(ConfigKeys.SECONDS_HANG_DETECTION, DefaultValues.SEC_HANG_DETECTION)
        self.auto_worker_enabled = _env("auto_worker_enabled", False)
        self.auto_ps_enabled = _env("auto_ps_enabled", False)
        self.relaunch_always = _env("relaunch_always", False)
        self.master_port = None

    @classmethod
    def singleton_instance(cls) -> "Context":
        with cls._lock:
            if cls._instance is None:
                cls._instance = cls()
            return cls._instance

    def config_master_port(self, port: int = 0):
        """Pick the master port from ``HOST_PORTS`` if given, else ``port``."""
        from .rpc import find_free_port, find_free_port_in_set

        hp = os.getenv("HOST_PORTS", "")
        if hp:
            try:
                self.master_port = find_free_port_in_set([int(p) for p in hp.split(",") if p])
                return self.master_port
            except RuntimeError:
                pass
        self.master_port = port or find_free_port()
        return self.master_port
