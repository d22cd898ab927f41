"""examples/data_parallelism.py without the engine (CPU): the model of each dataset accepts its
input shape, and the shards of get_processing_data (the reference's function, :47-53) cover the
data exactly once, the last rank taking the remainder."""
import importlib.util
import os

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
