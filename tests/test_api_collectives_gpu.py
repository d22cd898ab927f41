"""Broadcast / allgather operator surface at world size 1 on the GPU (tensor_communicate.py:9-129
mirrors): synchronous and keyed forms, sparse gradients, the data-parallel callbacks. At size 1
broadcast returns the tensor and allgather the tensor itself (concatenation of one block); the
keyed forms run the full fused pack -> collective -> unpack path."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope='module')
def world(gpu):
    from ddl.torch.communicator import Communicator
    return Communicator.world()


def test_broadcast_sync(world):
    from ddl.torch.tensor_communicate import broadcast, broadcast_
    x = torch.randn(333, 5, device='cuda')
    y = broadcast(x, 0, world)
    assert y.data_ptr() != x.data_ptr() and torch.equal(x, y)
    z = broadcast(x.cpu(), 0, world)
    assert not z.is_cuda and torch.equal(z, x.cpu())
    assert broadcast_(x, 0, world) is x
    with pytest.raises(Exception):
        broadcast(x, 1, world)  # root outside the world


@pytest.mark.parametrize('shape', [(7,), (0, 3), (1000, 3, 2), ()])
def test_allgather_sync(world, shape):
    from ddl.torch.tensor_communicate import allgather
    x = torch.randn(shape, device='cuda')
    y = allgather(x, world)
    assert torch.equal(y, x.reshape(-1, *x.shape[1:]) if x.dim() else x.reshape(1))


def test_allgather_int_and_host(world):
    from ddl.torch.tensor_communicate import allgather
    x = torch.arange(12, dtype=torch.int64).reshape(4, 3)
    assert torch.equal(allgather(x, world), x)


def test_keyed_broadcast_fused(world, lib):
    from ddl.torch.tensor_communicate import broadcast_async
    old = lib.ddl_get_config(b'fusion_threshold_bytes')
    lib.ddl_set_config(b'fusion_threshold_bytes', 10_000)  # several plans, some fused
    try:
        xs = [torch.randn(n, device='cuda') for n in (1, 700, 3000, 5, 2500)]
        hs = [broadcast_async(x, f'b{i}', 0, world) for i, x in enumerate(xs)]
        for x, h in zip(xs, hs):
            assert torch.equal(h.wait(), x)
    finally:
        lib.ddl_set_config(b'fusion_threshold_bytes', old)


def test_keyed_allgather_fused(world):
    """Several pending allgathers of one dtype: packed, gathered, unpacked (the m > 1 path of
    allgatherRequests) — each output equals its input at size 1."""
    from ddl.torch.tensor_communicate import allgather_async
    xs = [torch.randn(r, 3, device='cuda') for r in (4, 0, 9, 1)] + [torch.randn(6, device='cuda')]
    hs = [allgather_async(x, f'g{i}', world) for i, x in enumerate(xs)]
    for x, h in zip(xs, hs):
        y = h.wait()
        assert y.shape == x.shape and torch.equal(y, x)


def test_keyed_mixed_types_same_key(world):
    """The same key may be pending as an allreduce and a broadcast at once: requests are
    identified by (type, key) (RingTokenCommunicateHandler.cc:334)."""
    from ddl.torch.tensor_communicate import allgather_async, allreduce_async, broadcast_async
    x = torch.randn(100, device='cuda')
    h1 = allreduce_async(x, 'same', world)
    h2 = broadcast_async(x, 'same', 0, world)
    h3 = allgather_async(x, 'same', world)
    assert torch.equal(h1.wait(), x) and torch.equal(h2.wait(), x) and torch.equal(h3.wait(), x)


def test_sparse_gradient_allgather(world):
    from ddl.torch.tensor_communicate import allreduce_gradient
    i = torch.tensor([[0, 2, 2, 5]], device='cuda')
    v = torch.randn(4, 3, device='cuda')
    g = torch.sparse_coo_tensor(i, v, (8, 3))
    out = allreduce_gradient(g, world)
    assert out.is_sparse and out.shape == g.shape
    assert torch.equal(out.to_dense(), g.to_dense())


def test_broadcast_parameters_and_callbacks(world):
    from ddl.torch.parallelism.data import InitialParametersBroadcast, MetricAverage
    m = torch.nn.Sequential(torch.nn.Linear(8, 4), torch.nn.BatchNorm1d(4)).cuda()
    opt = torch.optim.Adam(m.parameters())
    m(torch.randn(16, 8, device='cuda')).sum().backward()
    opt.step()
    before = {k: v.clone() for k, v in m.state_dict().items()}
    cb = InitialParametersBroadcast(m, 0, opt, world)
    cb.on_batch_begin(0)
    for k, v in m.state_dict().items():
        assert torch.equal(v, before[k])
    logs = {'loss': 0.25, 'acc': 0.5}
    assert MetricAverage(world).on_epoch_end(0, dict(logs)) == logs  # size 1: unchanged
    assert MetricAverage(world).average(dict(logs)) == logs
