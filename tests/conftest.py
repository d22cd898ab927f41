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


def source_hash():
    """sha1 (16 hex) of the engine sources as the Makefile computes it for ddl_build_info()."""
    import glob
    import hashlib
    csrc = os.path.join(PKG, 'csrc')
    names = sorted(os.path.basename(f) for pat in ('*.h', '*.cpp', '*.hip') for f in glob.glob(os.path.join(csrc, pat)))
    h = hashlib.sha1()
    for f in [os.path.join(csrc, n) for n in names] + [os.path.join(ROOT, 'include', h) for h in ('ddl_amd.h', 'ddl_amd_testing.h')]:
        with open(f, 'rb') as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]


def _library_build_id(path):
    """The source hash baked into the library, read from the file (loading it here, before torch,
    would bind the engine to a second HIP runtime)."""
    import re
    try:
        with open(path, 'rb') as fh:
            m = re.search(rb'src=([0-9a-f]{16}) arch=gfx950', fh.read())
    except OSError:
        return None
    return m.group(1).decode() if m else None


DEPLOYMENT_LIB = os.path.join(PKG, 'lib', 'libddl_amd.so')
TESTING_LIB = os.path.join(PKG, 'lib', 'libddl_amd_testing.so')


def _build_if_stale():
    """The libraries under test must be built from these sources: built when missing, rebuilt
    when a baked-in source hash differs (a stale prebuilt .so is never tested)."""
    ora = os.path.join(ROOT, 'oracle', 'build', 'libddl_oracle.so')
    want = source_hash()
    if any(not os.path.exists(p) or _library_build_id(p) != want for p in (DEPLOYMENT_LIB, TESTING_LIB)):
        subprocess.run(['make', '-C', os.path.join(PKG, 'csrc'), '-j8', '-B'], check=True)
    if not os.path.exists(ora):
        subprocess.run(['make', '-C', os.path.join(ROOT, 'oracle')], check=True)


_build_if_stale()
# the suite drives the engine through the testing build (the same engine objects plus the test /
# measurement surface, include/ddl_amd_testing.h) via the reference's `ddl_lib` override; worker
# processes inherit it. tests/test_deployment_lib_gpu.py runs the deployment library on its own.
os.environ.setdefault('ddl_lib', TESTING_LIB)


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
