"""The RCCL transport on one GPU (ddl_rccl_loopback_*): a one-rank RCCL communicator, created by
the calls ddl_init makes at size > 1 (ncclGetUniqueId, ncclCommInitRank), carries the matched
send/recv pairs of P virtual ranks' programs as self-send / self-recv pairs through the
engine's RcclTransport::group — the code that replaces MPI_Allreduce at the reference's data
plane (MPICommunicator.cc:14-28). Also ncclCommSplit (MPICommunicator.cc:92-101) and the
autotuner's agreement (ncclAllReduce(MAX)) at size 1.

Bar: bit-exact vs the oracle — MPICH 3.3.2's order (ddlo_fold_ref_order) with reference_order
(default), the ring-order restatement with reference_order 0, MPI_Bcast / MPI_Allgatherv
restatements for the data-movement collectives — at P = 3, 5, 8, fp32 / fp64 / int32 / int64 /
uint64, on both sides of MPICH's 2048-byte switch, in and out of place, every schedule; P = 17,
20, 33 for the folds split beyond 16 inputs."""
import ctypes

import numpy as np
import pytest
import torch

from _helpers import (DT_DOUBLE, DT_FLOAT, DT_HALF, DT_INT32, DT_INT64, DT_UINT64, NAME, config, random_input,
                      ring_perms, ring_shape)

pytestmark = pytest.mark.gpu


@pytest.fixture(scope='module')
def loop(lib, gpu):
    st = lib.ddl_rccl_loopback_init(0)
    assert st == 0, lib.ddl_last_error()
    yield lib
    assert lib.ddl_rccl_loopback_finalize() == 0, lib.ddl_last_error()


def _dev(x, dev):
    return torch.from_numpy(np.ascontiguousarray(x).view(np.int16) if x.dtype == np.uint16 else x).to(dev)


def run_loop(lib, dev, xs, dt, in_place=False):
    ins = [_dev(x, dev) for x in xs]
    outs = ins if in_place else [torch.empty_like(t) for t in ins]
    P = len(xs)
    send = (ctypes.c_void_p * P)(*[t.data_ptr() for t in ins])
    recv = (ctypes.c_void_p * P)(*[t.data_ptr() for t in outs])
    st = lib.ddl_rccl_loopback_allreduce(P, send, recv, xs[0].size, dt, torch.cuda.current_stream().cuda_stream)
    assert st == 0, lib.ddl_last_error()
    torch.cuda.synchronize()
    return [o.cpu().numpy().view(xs[0].dtype) for o in outs]


def _pairs(lib, P):
    v = ctypes.c_longlong(-1)
    assert lib.ddl_rccl_loopback_stats(P, ctypes.byref(v)) == 0, lib.ddl_last_error()
    return v.value


@pytest.mark.parametrize('P', [3, 5, 8])
@pytest.mark.parametrize('dt', [DT_FLOAT, DT_DOUBLE, DT_INT32, DT_INT64, DT_UINT64], ids=lambda d: NAME[d])
@pytest.mark.parametrize('algo', [0, 1, 2, 3, 4])
def test_rccl_loopback_reference_order(loop, oracle, gpu, P, dt, algo):
    """Default reference order over the RCCL transport: every rank equals MPICH's order bit for
    bit, for messages up to 2048 bytes (binomial tree) and above (pre-fold + pairwise tree)."""
    lib = loop
    before = _pairs(lib, P)
    with config(lib, algo=algo, reference_order=1, tune=0, slice_bytes=64 << 10):
        for n in (1, 300, 4099, 300_001, 128 * 840):  # the last: equal chunks (direct-gather)
            xs = [random_input(dt, n, 17 * algo + 1234 + 7919 * r + n) for r in range(P)]
            want = oracle.fold_ref_order(dt, xs)
            for in_place in (False, True):
                for r, o in enumerate(run_loop(lib, gpu, xs, dt, in_place)):
                    assert o.tobytes() == want.tobytes(), (n, in_place, r)
    assert _pairs(lib, P) > before  # the bytes really went through RCCL


@pytest.mark.parametrize('P', [17, 20, 33])
@pytest.mark.parametrize('dt', [DT_FLOAT, DT_DOUBLE], ids=lambda d: NAME[d])
@pytest.mark.parametrize('algo', [1, 2, 3])
def test_rccl_loopback_reference_order_beyond_16(loop, oracle, gpu, P, dt, algo):
    """More than 16 ranks over the RCCL transport: the fold is split into <= 16-input steps
    through staging partials (plan_fold: MPICH's trees restricted to aligned blocks) and still
    equals MPICH's order bit for bit on every rank — both sides of the 2048-byte switch."""
    lib = loop
    with config(lib, algo=algo, reference_order=1, tune=0, slice_bytes=64 << 10):
        for n in (3, 300, 4099, 70_001):
            xs = [random_input(dt, n, 31 * algo + 555 + 7919 * r + n) for r in range(P)]
            want = oracle.fold_ref_order(dt, xs)
            for r, o in enumerate(run_loop(lib, gpu, xs, dt)):
                assert o.tobytes() == want.tobytes(), (n, r)


@pytest.mark.parametrize('P', [3, 5, 8])
@pytest.mark.parametrize('dt', [DT_FLOAT, DT_INT32, DT_HALF], ids=lambda d: NAME[d])
def test_rccl_loopback_ring_order(loop, oracle, gpu, P, dt):
    """The multi-ring schedule itself (reference_order 0) over RCCL: equals the ring-order
    restatement bit for bit (fp16 included: one rounding per hop)."""
    lib = loop
    with config(lib, algo=0, reference_order=0, tune=0, slice_bytes=256 << 10):
        for n in (257, 65_537, 1_000_003):
            xs = [random_input(dt, n, 99 + 7919 * r + n) for r in range(P)]
            R, _ = ring_shape(lib, n, dt, P)
            want = oracle.allreduce_ring(dt, xs, ring_perms(lib, P, R))
            for o in run_loop(lib, gpu, xs, dt):
                assert o.tobytes() == want.tobytes(), n


def test_rccl_loopback_c3_size(loop, oracle, gpu):
    """C3's shape through RCCL: 8 x 256 MiB random fp32, default schedule and order, against
    ddlo_fold_ref_order on every rank."""
    lib = loop
    P, n = 8, 64 << 20
    xs = [random_input(DT_FLOAT, n, 4242 + r) for r in range(P)]
    want = oracle.fold_ref_order(DT_FLOAT, xs)
    with config(lib, tune=0):
        outs = run_loop(lib, gpu, xs, DT_FLOAT, in_place=True)
    for r, o in enumerate(outs):
        assert o.tobytes() == want.tobytes(), r


@pytest.mark.parametrize('P', [3, 8])
def test_rccl_loopback_broadcast_allgatherv(loop, oracle, gpu, P):
    lib = loop
    s = torch.cuda.current_stream().cuda_stream
    n = 100_003
    xs = [random_input(DT_FLOAT, n, 5 + r) for r in range(P)]
    for root in (0, P - 1):
        bufs = [_dev(x, gpu) for x in xs]
        arr = (ctypes.c_void_p * P)(*[b.data_ptr() for b in bufs])
        assert lib.ddl_rccl_loopback_broadcast(P, root, arr, n, DT_FLOAT, s) == 0, lib.ddl_last_error()
        torch.cuda.synchronize()
        want = oracle.broadcast(DT_FLOAT, xs, root)
        for b, w in zip(bufs, want):
            assert b.cpu().numpy().tobytes() == w.tobytes()
    counts = [1000 * (q + 1) + q for q in range(P)]
    sends = [random_input(DT_INT32, c, 50 + q) for q, c in enumerate(counts)]
    displs = list(np.cumsum([0] + counts[:-1]))
    want = oracle.allgatherv(DT_INT32, sends, displs)
    ds = [_dev(x, gpu) for x in sends]
    rs = [torch.zeros(sum(counts), dtype=torch.int32, device=gpu) for _ in range(P)]
    Sz = ctypes.c_size_t * P
    assert lib.ddl_rccl_loopback_allgatherv(P, (ctypes.c_void_p * P)(*[d.data_ptr() for d in ds]),
                                            (ctypes.c_void_p * P)(*[r.data_ptr() for r in rs]), Sz(*counts),
                                            Sz(*[int(d) for d in displs]), DT_INT32, s) == 0, lib.ddl_last_error()
    torch.cuda.synchronize()
    for r in rs:
        assert r.cpu().numpy().tobytes() == want.tobytes()


def test_rccl_loopback_ncclallgather_call(loop, gpu):
    """RcclTransport::allgather — the gather-fold schedule's ncclAllGather — at one rank: the
    block lands at offset 0 of recv, nothing beyond it is touched."""
    lib = loop
    x = torch.arange(1001, dtype=torch.int32, device=gpu)
    y = torch.full((1100,), -7, dtype=torch.int32, device=gpu)
    assert lib.ddl_rccl_loopback_allgather(x.data_ptr(), y.data_ptr(), 1001 * 4,
                                           torch.cuda.current_stream().cuda_stream) == 0, lib.ddl_last_error()
    torch.cuda.synchronize()
    assert torch.equal(y[:1001], x) and bool((y[1001:] == -7).all())


def test_rccl_loopback_tuner_agreement(loop, gpu):
    """The autotuner's agreement step (ncclAllReduce(MAX), as Communicator::tune_ issues it) and
    a whole tuning pass with every candidate over RCCL: at one rank the max is the identity, the
    pick is a valid candidate, and the tuned schedule still sums exactly."""
    lib = loop
    s = torch.cuda.current_stream().cuda_stream
    vals = (ctypes.c_float * 5)(3.5, -1.0, 0.0, 7.25, 1e-3)
    assert lib.ddl_rccl_loopback_max(vals, 5, s) == 0, lib.ddl_last_error()
    assert list(vals) == [3.5, -1.0, 0.0, 7.25, np.float32(1e-3)]
    chosen, count = ctypes.c_int(-1), ctypes.c_int(0)
    cfgs, tms = (ctypes.c_longlong * 64)(), (ctypes.c_float * 16)()
    assert lib.ddl_rccl_loopback_tune(8, 1 << 18, DT_FLOAT, s, ctypes.byref(chosen), ctypes.byref(count), cfgs, tms,
                                      16) == 0, lib.ddl_last_error()
    assert count.value >= 2 and 0 <= chosen.value < count.value
    assert all(tms[i] > 0 for i in range(min(count.value, 16)))


def test_rccl_loopback_tuner_offers_sliced_c4_folds(loop, oracle, gpu):
    """a 16 MiB fp16 bucket at P = 8 (C4's, 2 MiB chunks) is tuned over
    direct candidates that cut each chunk into 4 and 8 slices (512 / 256 KiB), so a slice's fold
    can overlap the next slice's reduce-scatter; every candidate, run with the tuner off, sums
    bit-exact vs the oracle's fp16 rule (MPICH order in fp32, one rounding)."""
    lib = loop
    P, n = 8, (16 << 20) // 2
    s = torch.cuda.current_stream().cuda_stream
    chosen, count = ctypes.c_int(-1), ctypes.c_int(0)
    cfgs, tms = (ctypes.c_longlong * 128)(), (ctypes.c_float * 32)()
    assert lib.ddl_rccl_loopback_tune(P, n, DT_HALF, s, ctypes.byref(chosen), ctypes.byref(count), cfgs, tms,
                                      32) == 0, lib.ddl_last_error()
    cands = [tuple(cfgs[4 * i:4 * i + 4]) for i in range(min(count.value, 32))]
    direct = {c[2] for c in cands if c[0] == 1}
    assert {512 << 10, 256 << 10} <= direct, cands
    xs = [random_input(DT_HALF, n, 900 + r) for r in range(P)]
    want = oracle.fold_ref_order(DT_HALF, xs).tobytes()
    for slice_bytes in (512 << 10, 256 << 10):
        with config(lib, tune=0, algo=1, slice_bytes=slice_bytes, max_slices=16):
            for o in run_loop(lib, gpu, xs, DT_HALF):
                assert o.tobytes() == want, slice_bytes


def test_rccl_loopback_split(loop, oracle, gpu):
    """ncclCommSplit at size 1 (the handler's private data communicator and every
    split_communicator go through it): color 0 gives rank 0 of 1, and the split communicator
    carries the transport bit-exactly; a negative color leaves the rank in no communicator."""
    lib = loop
    r, s = ctypes.c_int(-5), ctypes.c_int(-5)
    assert lib.ddl_rccl_loopback_split(-1, 0, ctypes.byref(r), ctypes.byref(s)) == 0, lib.ddl_last_error()
    assert (r.value, s.value) == (-1, 0)
    assert lib.ddl_rccl_loopback_split(0, 0, ctypes.byref(r), ctypes.byref(s)) == 0, lib.ddl_last_error()
    assert (r.value, s.value) == (0, 1)
    P, n = 5, 4099
    xs = [random_input(DT_DOUBLE, n, 321 + q) for q in range(P)]
    with config(lib, tune=0):
        for o in run_loop(lib, gpu, xs, DT_DOUBLE):
            assert o.tobytes() == oracle.fold_ref_order(DT_DOUBLE, xs).tobytes()
    assert _pairs(lib, P) > 0
