"""Framework-wide constants.

Parity notes: mirrors the enum families of the reference
``dlrover/python/common/constants.py`` (NodeEnv :205-231, RendezvousName :263,
TrainingExceptionLevel :278, ConfigPath :286-291, CheckpointConstant :294-298,
Accelerators :301).  Values that users may already have in their job specs
(environment-variable names, tracker-file names) are kept identical so that a
job written for the reference keeps working.
"""


class NodeType:
    WORKER = "worker"
    MASTER = "master"
    CHIEF = "chief"
    PS = "ps"
    EVALUATOR = "evaluator"


class PSClusterVersionType:
    GLOBAL = "GLOBAL"
    LOCAL = "LOCAL"
    RESTORED = "RESTORED"


class NodeStatus:
    INITIAL = "Initial"
    PENDING = "Pending"
    RUNNING = "Running"
    SUCCEEDED = "Succeeded"
    FAILED = "Failed"
    DELETED = "Deleted"
    FINISHED = "Finished"
    BREAKDOWN = "Breakdown"
    UNKNOWN = "Unknown"


class NodeEventType:
    ADDED = "ADDED"
    MODIFIED = "MODIFIED"
    DELETED = "DELETED"
    ERROR = "ERROR"


class NodeExitReason:
    SUCCEEDED = "Succeeded"
    KILLED = "Deleted"
    OOM = "OOMKilled"
    FATAL_ERROR = "Error"
    HARDWARE_ERROR = "HardwareError"
    NO_HEARTBEAT = "NoHeartBeat"
    UNKNOWN_ERROR = "UnknownError"


class JobExitReason:
    SUCCEEDED = "Completed"
    CODE_ERROR = "CodeError"
    WORKER_OOM = "WorkerOOM"
    WORKER_ERROR = "WorkerError"
    HANG_ERROR = "HangError"
    RDZV_TIMEOUT_ERROR = "RdzvTimeout"
    PENDING_TIMEOUT = "PendingTimeout"
    UNKNOWN_ERROR = "UnknownError"


class DistributionStrategy:
    LOCAL = "Local"
    PS = "ParameterServerStrategy"
    ALLREDUCE = "AllreduceStrategy"
    CUSTOM = "CustomStrategy"


class GRPC:
    MAX_SEND_MESSAGE_LENGTH = 256 * 1024 * 1024
    MAX_RECEIVE_MESSAGE_LENGTH = 256 * 1024 * 1024


class TrainingLoopStatus:
    START = 1
    END = 2
    PENDING = 3


class NodeEnv:
    """Environment variable names (identical to the reference)."""

    RELAUNCHED_POD = "RELAUNCHED_POD"
    DLROVER_MASTER_ADDR = "DLROVER_MASTER_ADDR"
    GRPC_ENABLE_FORK = "GRPC_ENABLE_FORK_SUPPORT"
    POD_NAME = "POD_NAME"
    MONITOR_ENABLED = "MONITOR_ENABLED"
    JOB_NAME = "ELASTIC_JOB_NAME"
    JOB_UID = "JOB_UID"
    NODE_TYPE = "NODE_TYPE"
    NODE_ID = "NODE_ID"
    NODE_NUM = "NODE_NUM"
    NODE_RANK = "NODE_RANK"
    WORKER_TYPE = "WORKER_TYPE"
    WORKER_ID = "WORKER_ID"
    WORKER_NUM = "WORKER_NUM"
    WORKER_RANK = "WORKER_RANK"
    RANK = "RANK"
    WORLD_SIZE = "WORLD_SIZE"
    TORCHELASTIC_RUN_ID = "TORCHELASTIC_RUN_ID"
    # Fault injection used by node-check and the goodput benchmark.
    MOCK_ERR_RANK = "MOCK_ERR_RANK"
    FAULT_INJECT_STEP = "DWAMD_FAULT_INJECT_STEP"
    FAULT_INJECT_RANK = "DWAMD_FAULT_INJECT_RANK"


class DatasetType:
    TEXT = "text"
    MAXCOMPUTE_TABLE = "maxcompute_table"


class RendezvousName:
    ELASTIC_TRAINING = "elastic-training"
    NETWORK_CHECK = "network-check"


class NodeErrorMessage:
    NETWORKER_ERROR = "Network is breakdown"
    SOCKET_GAIERROR = "Name or service not known"


class NetworkFailureReason:
    NODE_FAILURE = "Node Failure"
    WAITING_NODE = "Waiting node"


class TrainingExceptionLevel:
    RDZV_ERROR = "rdzv_error"
    PROCESS_ERROR = "process_error"
    NODE_ERROR = "node_error"
    WARNING = "warning"
    INFO = "info"


class ConfigPath:
    ENV_PARAL_CONFIG = "DLROVER_PARAL_CONFIG_PATH"
    PARAL_CONFIG = "/tmp/dlrover/auto_paral_config.json"
    ENV_RUNTIME_METRICS = "RUNTIME_METRICS_PATH"
    RUNTIME_METRICS = "/tmp/dlrover/runtime_metrics.json"
    NETWORK_CHECK_DATA_DIR = "/tmp/dlrover/network_check/"


class CheckpointConstant:
    TRACER_FILE_NAME = "dlrover_latest.txt"
    MODEL_STATES_NAME = "model_states"
    OPTIM_STATES_NAME = "optim_states"
    SAVE_TIMEOUT = 600


class Accelerators:
    AMD_GPU = "amd.com/gpu"
    NVIDIA_GPU = "nvidia.com/gpu"  # accepted on the CLI, mapped to AMD_GPU
    ASCEND_NPU = "ascend-npu"
    CPU = "cpu"


class JobConstant:
    RDZV_JOIN_TIMEOUT_DEFAULT = 600
    RDZV_POLL_INTERVAL = 1.0
    HEARTBEAT_INTERVAL = 15
    MASTER_CLIENT_TIMEOUT = 5
    MASTER_CLIENT_RETRY = 10
    TRAINING_AGENT_LOOP_INTERVAL = 0.5
    NODE_HEARTBEAT_TIMEOUT = 300
    MAX_RESTART_DEFAULT = 3


class CommBackend:
    """RCCL is exposed by torch.distributed under the name ``nccl``."""

    RCCL = "nccl"
    GLOO = "gloo"


class NodeResourceLimit:
    """Bounds for automatic resource adjustment (reference constants.py:131).
    Memory in MiB.  MI355X hosts carry far more RAM than the reference's CPU
    pods: the OOM bump ceiling is sized for a GPU node's host memory."""

    MAX_CPU_CORES = 256
    MIN_CPU_CORES = 4
    MIN_MEMORY = 6144
    MAX_MEMORY = 2 * 1024 * 1024  # 2 TiB
    INCREMENTAL_MEMORY_FACTOR = 2
    MAX_INCREMENTAL_MEMORY = 256 * 1024  # one OOM relaunch adds at most 256 GiB
