import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, 'experiment-distributed-deep-learning_amd')
TESTS = os.path.dirname(os.path.abspath(__file__))
for p in (PKG, TESTS, ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line('markers', 'gpu: needs an MI355X (runs on the GPU box)')
    config.addinivalue_line('markers', 'slow: longer CPU test')


def _build_if_missing():
    lib = os.path.join(PKG, 'lib', 'libddl_amd.so')
    ora = os.path.join(ROOT, 'oracle', 'build', 'libddl_oracle.so')
    if not os.path.exists(lib):
        subprocess.run(['make', '-C', os.path.join(PKG, 'csrc'), '-j8'], check=True)
    if not os.path.exists(ora):
        subprocess.run(['make', '-C', os.path.join(ROOT, 'oracle')], check=True)


_build_if_missing()


@pytest.fixture(scope='session')
def lib():
    from ddl.torch.cpp_backend import CPPBackend
    return CPPBackend.c_api()


@pytest.fixture(scope='session')
def oracle():
    import _helpers
    return _helpers.Oracle()


@pytest.fixture(scope='session')
def gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.skip('no GPU')
    torch.cuda.set_device(0)
    return torch.device('cuda', 0)
