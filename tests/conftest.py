import os
import sys

import pytest

# torch first: its bundled HIP runtime and the system ROCm one libgwa.so links share the SONAME
# libamdhip64.so.7, so whichever a process loads first serves both; torch initialises its device only
# on its own runtime.  The GPU tests that hand SAM text to torch tensors (dist.gather_sam_device) need
# torch loaded before libgwa, as bench.py does.
import torch  # noqa: E402,F401

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "oracle"))
sys.path.insert(0, os.path.join(REPO, "genome-weaver-align_amd"))
sys.path.insert(0, REPO)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (run on the GPU box via gpurun)")
    config.addinivalue_line("markers", "slow: long-running CPU test")
