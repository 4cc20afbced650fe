import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
HERE = os.path.dirname(os.path.abspath(__file__))
if HERE not in sys.path:
    sys.path.insert(0, HERE)


def pytest_configure(config):
    config.addinivalue_line('markers', 'gpu: needs a ROCm GPU (MI355X) and the built libsphrt.so')
    config.addinivalue_line('markers', 'slow: large sizes (full BASELINE configs)')


@pytest.fixture(scope='session')
def gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.fail('GPU test requested but torch.cuda.is_available() is False')
    from sph_raytracer_amd import build
    build.build()
    return torch.device('cuda', 0)
