"""Which GPUs does this process hold open (DRM fdinfo drm-pdev), and what do
the amdgpu sysfs counters of those GPUs say?  (elastic_agent/monitor.py
process_gpu_pdevs / gpu_stats on a real box.)"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from dlrover_wuqiong_amd.elastic_agent.monitor import ResourceMonitor  # noqa: E402

x = torch.empty(1 << 30, dtype=torch.uint8, device="cuda")
torch.cuda.synchronize()
pd = ResourceMonitor.process_gpu_pdevs([os.getpid()])
print("pdevs:", sorted(pd))
print("all gpus:", [(g.index, g.used_memory_mb, g.total_memory_mb) for g in ResourceMonitor.gpu_stats()])
print("job gpus:", [(g.index, g.used_memory_mb, g.total_memory_mb) for g in ResourceMonitor.gpu_stats(pd)])
