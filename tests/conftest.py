import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "sph-exa_amd", "python")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs via gpurun on the GPU box)")
    config.addinivalue_line("markers", "ref: needs oracle/_ref (the reference built from /root/reference)")
    config.addinivalue_line("markers", "slow: longer CPU test")
