"""Packaging for ``pip install [-e] .``: the ``det`` CLI, master and agent entry points, the
in-tree HIP/C++ sources and built extensions (build them for gfx950 first:
``python -c "import __graft_entry__ as g; g.build()"``), and the web UI."""
from setuptools import find_packages, setup

setup(
    name="determined_clone_amd",
    version="0.1.0",
    description=("MI355X-native deep-learning training platform: Core API / PyTorchTrial / "
                 "DeepSpeedTrial harness, master + agent, det CLI, HIP/CDNA4 kernels, RCCL "
                 "data / ZeRO / pipeline parallelism"),
    python_requires=">=3.10",
    packages=find_packages(include=["determined_clone_amd", "determined_clone_amd.*"]),
    package_data={
        "determined_clone_amd.ops": ["csrc/*", "*.so", "tuned/*.csv", "tuned/miopen/db/*",
                                     "tuned/miopen/cache/*"],
        "determined_clone_amd.native": ["*.cpp", "*.so", "bin/*"],
        "determined_clone_amd.webui": ["static/*"],
    },
    install_requires=["torch", "numpy", "pyyaml", "requests", "psutil"],
    entry_points={"console_scripts": [
        # `det` is the reference's CLI; master / agent stand in for determined-master / -agent
        "det = determined_clone_amd.cli.cli:main",
        "det-clone-master = determined_clone_amd.master.__main__:main",
        "det-clone-agent = determined_clone_amd.agent.agent:main",
        "det-dsat = determined_clone_amd.pytorch.dsat.__main__:main",
    ]},
)
