"""Package metadata: `pip install -e .` (editable -- the gfx950 extension is compiled in-tree,
fedmi/ops/_fedmi_hip*.so, on first use or with `fedmi-build`; fedmi.ops.native() refuses a binary
whose compiled-in source digest does not match the sources next to it)."""
from setuptools import find_packages, setup

setup(
    name="fedmi",
    version="0.4.0",
    description="MI355X-native federated learning: fused gfx950 HIP round kernels, FedAvg over xGMI / RCCL",
    long_description=open("README.md", encoding="utf-8").read(),
    long_description_content_type="text/markdown",
    python_requires=">=3.10",
    packages=find_packages(include=["fedmi", "fedmi.*"]),
    package_data={"fedmi.ops": ["csrc/*.hip", "csrc/*.h", "csrc/*.inc", "csrc/*.cpp"]},
    install_requires=["torch>=2.4", "numpy", "safetensors", "pybind11"],
    extras_require={"sklearn": ["scikit-learn"], "test": ["pytest", "pytest-timeout"]},
    entry_points={"console_scripts": ["fedmi-build = fedmi.ops.build:main"]},
)
