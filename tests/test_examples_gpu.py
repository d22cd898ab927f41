"""examples/data_parallelism.py — the torch counterpart of the reference's DP script
(src/py/ddl/examples/data_parallelism.py) — runs as a training script would: a fresh process, the
deployment library only (no `ddl_lib` override), one rank (the pool's boxes have one GPU; the
multi-rank form of the same calls is tests/_mp_gpu_worker.check_dp_training). It trains on its
synthetic MNIST-shaped data, the learning rate warms up, and the loss falls."""
import os
import re
import subprocess
import sys

import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu


def test_data_parallelism_example_trains():
    env = dict(os.environ)
    env.pop('ddl_lib', None)
    p = subprocess.run([sys.executable, os.path.join(ROOT, 'examples', 'data_parallelism.py'), '--epochs', '3',
                        '--samples', '4096', '--warmup_epochs', '2', '--lr', '0.002'],
                       env=env, capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, p.stderr[-3000:]
    losses = [float(m) for m in re.findall(r'loss ([0-9.e+-]+)', p.stdout)]
    lrs = [float(m) for m in re.findall(r'lr ([0-9.e+-]+)', p.stdout)]
    assert len(losses) == 3 and losses[-1] < losses[0], p.stdout
    assert lrs[1] == pytest.approx(0.002, rel=1e-6)  # warmed up to the (size-scaled) lr after 2 epochs
    assert 'finished gradual learning rate warmup' in p.stdout


def test_c_example_runs_on_the_deployment_library(tmp_path):
    """examples/c_host_allreduce.c: C1's host allreduce, a keyed batch of host buckets completed
    through a completion group, a split — from C, linked against lib/libddl_amd.so alone; the
    one-rank data plane forced, every output checked bit for bit against its input."""
    from test_examples_cpu import build_c_example
    exe = build_c_example(tmp_path)
    env = dict(os.environ)
    env.pop('ddl_lib', None)
    p = subprocess.run([exe, '0'], env=env, capture_output=True, text=True, timeout=120)
    assert p.returncode == 0, (p.stdout, p.stderr[-3000:])
    assert 'c_host_allreduce: ok' in p.stdout
