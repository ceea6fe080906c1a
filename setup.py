"""Packaging: the framework plus the DLRover / ATorch import-path
compatibility packages, and the reference's console scripts
(reference setup.py:39-62: ``dlrover-run`` -> dlrover.trainer.torch.main)."""

from setuptools import find_packages, setup

setup(
    name="dlrover_wuqiong_amd",
    version="0.3.0",
    description="MI355X-native elastic training and flash checkpointing (DLRover / ATorch capabilities on "
                "PyTorch-ROCm, HIP/CDNA4 kernels and RCCL)",
    long_description=open("README.md").read() if __import__("os").path.exists("README.md") else "",
    long_description_content_type="text/markdown",
    python_requires=">=3.10",
    packages=find_packages(include=["dlrover_wuqiong_amd", "dlrover_wuqiong_amd.*", "dlrover", "dlrover.*",
                                    "atorch", "atorch.*"]),
    package_data={"dlrover_wuqiong_amd": ["_native/*.so", "csrc/kernels/*.hip", "csrc/kernels/*.h",
                                          "csrc/runtime/*.cpp", "csrc/runtime/*.h"]},
    install_requires=["torch", "numpy", "grpcio", "psutil", "pyyaml"],
    extras_require={"hf": ["transformers", "accelerate", "safetensors"], "ray": ["ray"]},
    entry_points={"console_scripts": [
        "dlrover-run = dlrover.trainer.torch.main:main",
        "dwamd-run = dlrover_wuqiong_amd.trainer.run:main",
        "dwamd-master = dlrover_wuqiong_amd.master.master:main",
        "dwamd-brain = dlrover_wuqiong_amd.brain.service:main",
        "dwamd-brain-k8s-monitor = dlrover_wuqiong_amd.brain.k8s_monitor:main",
        "dwamd-operator = dlrover_wuqiong_amd.platform.k8s:main",
    ]},
)
