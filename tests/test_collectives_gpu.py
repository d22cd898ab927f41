"""Broadcast and allgather on the GPU: the same per-rank programs the RCCL path runs, executed
by P virtual ranks on one GPU (ddl_local_broadcast / ddl_local_allgatherv: device copies stand
in for RCCL send/recv), bit-exact against the oracle's MPI_Bcast / MPI_Allgatherv."""
import ctypes

import numpy as np
import pytest
import torch

from _helpers import ALL_DTYPES, DT_FLOAT, NAME, SZ, config, random_input

pytestmark = pytest.mark.gpu


def dev_tensor(x, dev):
    return torch.from_numpy(x.view(np.int16) if x.dtype == np.uint16 else x).to(dev)


@pytest.mark.parametrize('P', [1, 2, 3, 4, 8])
@pytest.mark.parametrize('dt', ALL_DTYPES, ids=lambda d: NAME[d])
@pytest.mark.parametrize('n', [1, 4099, 1_000_003])
def test_local_broadcast(lib, oracle, gpu, P, dt, n):
    root = P - 1
    xs = [random_input(dt, n, 100 + r) for r in range(P)]
    ts = [dev_tensor(x, gpu) for x in xs]
    arr = (ctypes.c_void_p * P)(*[t.data_ptr() for t in ts])
    with config(lib, slice_bytes=256 << 10):
        st = lib.ddl_local_broadcast(P, root, arr, n, dt, torch.cuda.current_stream().cuda_stream)
        assert st == 0, lib.ddl_last_error()
        torch.cuda.synchronize()
    want = oracle.broadcast(dt, xs, root)
    for r in range(P):
        assert ts[r].cpu().numpy().tobytes() == want[r].tobytes(), r


def test_local_broadcast_full_size(lib, gpu):
    """256 MiB fp32 from rank 2 of 8 (K = 8 pipelined slices)."""
    P, n = 8, 64 << 20
    ts = [torch.full((n,), float(r), device=gpu) for r in range(P)]
    ts[2].copy_(torch.randn(n, device=gpu))
    arr = (ctypes.c_void_p * P)(*[t.data_ptr() for t in ts])
    assert lib.ddl_local_broadcast(P, 2, arr, n, DT_FLOAT, torch.cuda.current_stream().cuda_stream) == 0
    torch.cuda.synchronize()
    for t in ts:
        assert torch.equal(t, ts[2])


@pytest.mark.parametrize('P', [1, 2, 3, 8])
@pytest.mark.parametrize('dt', ALL_DTYPES, ids=lambda d: NAME[d])
def test_local_allgatherv(lib, oracle, gpu, P, dt):
    rng = np.random.default_rng(P + dt)
    counts = [int(c) for c in rng.integers(0, 200_000, size=P)]
    if P > 2:
        counts[2] = 0
    displs = list(np.cumsum([0] + counts[:-1]))
    total = sum(counts)
    xs = [random_input(dt, c, 300 + q) for q, c in enumerate(counts)]
    sends = [dev_tensor(x, gpu) for x in xs]
    recvs = [torch.zeros(total, dtype=s.dtype, device=gpu) for s in sends]
    S = (ctypes.c_void_p * P)(*[s.data_ptr() for s in sends])
    R = (ctypes.c_void_p * P)(*[r.data_ptr() for r in recvs])
    st = lib.ddl_local_allgatherv(P, S, R, (SZ * P)(*counts), (SZ * P)(*[int(d) for d in displs]), dt,
                                  torch.cuda.current_stream().cuda_stream)
    assert st == 0, lib.ddl_last_error()
    torch.cuda.synchronize()
    want = oracle.allgatherv(dt, xs)
    for r in range(P):
        assert recvs[r].cpu().numpy().tobytes() == want.tobytes(), r


def test_local_allgatherv_in_place(lib, oracle, gpu):
    """MPI_IN_PLACE style: each rank's contribution already sits at its displacement."""
    P, c = 4, 12_345
    xs = [random_input(DT_FLOAT, c, q) for q in range(P)]
    recvs = [torch.zeros(P * c, device=gpu) for _ in range(P)]
    for q in range(P):
        recvs[q][q * c:(q + 1) * c] = torch.from_numpy(xs[q]).to(gpu)
    S = (ctypes.c_void_p * P)(*[recvs[q].data_ptr() + 4 * q * c for q in range(P)])
    R = (ctypes.c_void_p * P)(*[r.data_ptr() for r in recvs])
    assert lib.ddl_local_allgatherv(P, S, R, (SZ * P)(*[c] * P), (SZ * P)(*[q * c for q in range(P)]), DT_FLOAT,
                                    torch.cuda.current_stream().cuda_stream) == 0
    torch.cuda.synchronize()
    want = np.concatenate(xs)
    for r in recvs:
        assert r.cpu().numpy().tobytes() == want.tobytes()


def test_world_broadcast_allgather_size1(lib, gpu):
    """The communicator entries at world size 1: broadcast leaves the buffer, allgather copies."""
    from ddl.torch.communicator import Communicator
    comm = Communicator.world()
    x = torch.randn(1000, device=gpu)
    y = x.clone()
    s = torch.cuda.current_stream().cuda_stream
    assert lib.ddl_broadcast(comm.id, y.data_ptr(), 1000, DT_FLOAT, 0, s) == 0
    out = torch.zeros(1000, device=gpu)
    assert lib.ddl_allgather(comm.id, x.data_ptr(), 1000, out.data_ptr(), 1000, DT_FLOAT, s) == 0
    torch.cuda.synchronize()
    assert torch.equal(y, x) and torch.equal(out, x)
    assert lib.ddl_broadcast(comm.id, y.data_ptr(), 1000, DT_FLOAT, 1, s) == 3  # root outside the world


@pytest.mark.parametrize('P', [4, 5, 8])
def test_reference_broadcast_known_answer(lib, gpu, P):
    """broadcast_test.py:5-17: fp32[16] = rank + 1 on every rank, broadcast from root 3 ->
    every rank holds 4."""
    ts = [torch.full((16,), float(r + 1), device=gpu) for r in range(P)]
    arr = (ctypes.c_void_p * P)(*[t.data_ptr() for t in ts])
    assert lib.ddl_local_broadcast(P, 3, arr, 16, DT_FLOAT, torch.cuda.current_stream().cuda_stream) == 0
    torch.cuda.synchronize()
    for t in ts:
        assert torch.all(t == 4.0)


@pytest.mark.parametrize('P', [2, 3, 4])
def test_reference_allgather_known_answer(lib, oracle, gpu, P):
    """allgather_test.py:5-26: IndexedSlices values = arange(4 + rank) + rank (first dims differ
    per rank), indices = [[0,0],[1,1],[2,2],[3,3]] + rank; both allgathered -> the rank-ordered
    concatenations (the keyed layout of MPIRingTokenCommunication.cc:338-356)."""
    values = [np.arange(4 + r, dtype=np.float32) + r for r in range(P)]
    indices = [(np.array([[0, 0], [1, 1], [2, 2], [3, 3]]) + r).astype(np.float32) for r in range(P)]
    for parts in (values, [x.reshape(-1) for x in indices]):
        counts = [x.size for x in parts]
        displs = list(np.cumsum([0] + counts[:-1]))
        sends = [torch.from_numpy(x).to(gpu) for x in parts]
        recvs = [torch.zeros(sum(counts), device=gpu) for _ in range(P)]
        S = (ctypes.c_void_p * P)(*[s.data_ptr() for s in sends])
        R = (ctypes.c_void_p * P)(*[r.data_ptr() for r in recvs])
        assert lib.ddl_local_allgatherv(P, S, R, (SZ * P)(*counts), (SZ * P)(*[int(d) for d in displs]), DT_FLOAT,
                                        torch.cuda.current_stream().cuda_stream) == 0
        torch.cuda.synchronize()
        want = np.concatenate(parts)
        for r in recvs:
            assert np.array_equal(r.cpu().numpy(), want)
    got = oracle.allgather_requests(DT_FLOAT, [[v, i] for v, i in zip(values, indices)])
    assert np.array_equal(got[0], np.concatenate(values))
    assert np.array_equal(got[1], np.concatenate(indices))
