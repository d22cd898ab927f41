"""examples/ without a GPU: data_parallelism.py's model of each dataset accepts its input shape,
and the shards of get_processing_data (the reference's function, :47-53) cover the data exactly
once, the last rank taking the remainder; c_host_allreduce.c, the reference's CPU op as a plain C
caller of the deployment header, compiles as C99 with every warning an error and links against
lib/libddl_amd.so alone, and without a GPU fails loudly (no CPU fallback)."""
import importlib.util
import os
import shutil
import subprocess

import pytest
import torch

from conftest import ROOT


def _example():
    spec = importlib.util.spec_from_file_location('dp_example', os.path.join(ROOT, 'examples', 'data_parallelism.py'))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


@pytest.mark.parametrize('dataset', ['mnist', 'cifar10'])
def test_models_take_their_shapes(dataset):
    m = _example()
    model, (c, hw) = m.model_for(dataset)
    x, y = m.synthetic(16, (c, hw, hw))
    assert model(x).shape == (16, 10) and y.shape == (16,) and int(y.max()) < 10


@pytest.mark.parametrize('size', [1, 3, 8])
def test_shards_cover_the_data(size):
    m = _example()

    class Comm:
        def __init__(self, rank):
            self.rank, self.size = rank, size
    data = torch.arange(1001)
    parts = [m.get_processing_data(data, Comm(r)) for r in range(size)]
    assert torch.equal(torch.cat(parts), data)
    assert all(len(p) == 1001 // size for p in parts[:-1])


def build_c_example(out_dir):
    """gcc -std=c99 -Werror against include/ddl_amd.h and lib/libddl_amd.so (the deployment
    library: every symbol the example uses must be in the header's export list)."""
    lib_dir = os.path.join(ROOT, 'experiment-distributed-deep-learning_amd', 'lib')
    exe = os.path.join(str(out_dir), 'c_host_allreduce')
    subprocess.run(['gcc', '-std=c99', '-Wall', '-Wextra', '-Werror', '-pedantic', '-I', os.path.join(ROOT, 'include'),
                    os.path.join(ROOT, 'examples', 'c_host_allreduce.c'), '-L', lib_dir, '-lddl_amd',
                    f'-Wl,-rpath,{lib_dir}', '-o', exe], check=True, capture_output=True, text=True)
    return exe


@pytest.mark.skipif(shutil.which('gcc') is None, reason='no C compiler')
def test_c_example_builds_against_the_deployment_header(tmp_path):
    exe = build_c_example(tmp_path)
    maps = subprocess.run(['ldd', exe], capture_output=True, text=True, check=True).stdout
    assert 'libddl_amd.so' in maps and 'libddl_amd_testing' not in maps
    if not torch.cuda.is_available():  # this container: the engine refuses to start, loudly
        p = subprocess.run([exe], capture_output=True, text=True, timeout=120)
        assert p.returncode == 1 and 'ddl_init_single' in p.stderr, (p.returncode, p.stderr)
