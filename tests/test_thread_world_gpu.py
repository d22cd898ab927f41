"""The production executor (RingExecutor, what ddl_allreduce runs at N > 1) driven ASYNCHRONOUSLY
at P = 2..8 on one GPU (VERDICT r2 missing #2 / next #2): P threads, each owning its own
RingExecutor, exchange through the in-process ThreadFabric with RCCL's contract — a group
rendezvous with its peers only on the host enqueue, a receive is a stream wait on the sender's
event plus a D2D copy, the sender's stream waits for the receiver's copy event, and nothing
synchronises the host (executor.h ThreadFabric). So the executor's own event chain between the
caller's stream, its comm stream and its compute stream is what keeps the data right: a missing
wait corrupts the sums here, where the host-synchronising test transport would hide it.

Bar: every rank bit-exact vs MPICH's order (ddlo_fold_ref_order) — or the ring-order / left-fold
restatements with reference_order 0 — on the MPICH golden vectors, the oracle cases and C3 at
full size (8 x 256 MiB), for every schedule; broadcast / allgatherv vs MPI_Bcast / MPI_Allgatherv
restatements. The mutation test drops ONE reduce wait (ddl_testing_drop_wait) and must see wrong
data (reference semantics: MPIRingTokenCommunication.cc:548-733, MPICommunicator.cc:14-28)."""
import ctypes
import json
import os

import numpy as np
import pytest
import torch

from _helpers import DT_DOUBLE, DT_FLOAT, DT_INT32, NAME, config, random_input, ring_perms, ring_shape

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
TORCH_DT = {np.dtype(np.float32): torch.float32, np.dtype(np.float64): torch.float64,
            np.dtype(np.int32): torch.int32, np.dtype(np.int64): torch.int64, np.dtype(np.uint64): torch.int64}


def _dev(x, gpu):
    return torch.from_numpy(np.ascontiguousarray(x).view(np.int64) if x.dtype == np.uint64 else x).to(gpu)


def _host(t, like):
    return t.cpu().numpy().view(like.dtype)


def _thread_allreduce(lib, ins, outs, n, dt):
    P = len(ins)
    send = (ctypes.c_void_p * P)(*[t.data_ptr() for t in ins])
    recv = (ctypes.c_void_p * P)(*[t.data_ptr() for t in outs])
    st = lib.ddl_testing_thread_allreduce(P, send, recv, n, dt, torch.cuda.current_stream().cuda_stream)
    assert st == 0, lib.ddl_last_error()


def _run(lib, gpu, xs, dt, in_place=False):
    ins = [_dev(x, gpu) for x in xs]
    outs = ins if in_place else [torch.full_like(t, -7) for t in ins]
    _thread_allreduce(lib, ins, outs, xs[0].size, dt)
    torch.cuda.synchronize()
    return [_host(o, xs[0]) for o in outs]


def _golden():
    gold = np.load(os.path.join(HERE, 'golden', 'golden_mpich.npz'), allow_pickle=False)
    meta = json.load(open(os.path.join(HERE, 'golden', 'golden_manifest.json')))['cases']
    return [(case, m, gold[case + '__inputs'], gold[case + '__output']) for case, m in meta.items()]


DT_OF = {np.dtype(np.float32): DT_FLOAT, np.dtype(np.float64): DT_DOUBLE, np.dtype(np.int32): DT_INT32,
         np.dtype(np.int64): 9, np.dtype(np.uint64): 23}


@pytest.mark.parametrize('algo', [0, 1, 2, 3, 4])
def test_thread_world_mpich_golden(lib, gpu, algo):
    """Every MPICH 3.3.2 golden case (P = 2..8, both sides of its 2048-byte switch) through the
    asynchronous executor, every schedule, in and out of place: bit for bit on every rank."""
    with config(lib, algo=algo, reference_order=1, tune=0, slice_bytes=64 << 10):
        for case, m, xs, y in _golden():
            for in_place in (False, True):
                for r, o in enumerate(_run(lib, gpu, list(xs), DT_OF[xs.dtype], in_place)):
                    assert o.tobytes() == y.tobytes(), (case, in_place, r)


@pytest.mark.parametrize('P', [2, 3, 5, 8])
@pytest.mark.parametrize('algo,ref', [(0, 0), (1, 0), (2, 0), (3, 0), (0, 1), (1, 1), (2, 1), (3, 1), (4, 1)])
@pytest.mark.parametrize('dt', [DT_FLOAT, DT_DOUBLE, DT_INT32], ids=lambda d: NAME[d])
def test_thread_world_schedules_vs_oracle(lib, oracle, gpu, P, algo, ref, dt):
    """Oracle cases with many slices per chunk (64 KiB slices: the recv / reduce / send overlap
    of the executor is exercised tick by tick)."""
    with config(lib, algo=algo, reference_order=ref, tune=0, slice_bytes=64 << 10):
        for n in (1, 300, 65_537, 1_000_003, 128 * 840):
            xs = [random_input(dt, n, 31 * algo + 7 * P + 1000 * ref + 13 * q + n) for q in range(P)]
            if ref:
                want = oracle.fold_ref_order(dt, xs)
            elif algo == 0:
                R, _ = ring_shape(lib, n, dt, P)
                want = oracle.allreduce_ring(dt, xs, ring_perms(lib, P, R))
            elif algo == 1:
                want = oracle.allreduce_direct(dt, xs)
            else:
                want = oracle.fold(dt, xs)
            for r, o in enumerate(_run(lib, gpu, xs, dt, in_place=(n % 2 == 1))):
                assert o.tobytes() == want.tobytes(), (n, r)


@pytest.mark.parametrize('algo', [1, 4])
def test_thread_world_c3_full_size(lib, oracle, gpu, algo):
    """C3: 8 x 256 MiB random fp32 per rank, the default reference-order schedule (direct; and
    direct-gather), 2 MiB slices — the N = 8 headline workload through the asynchronous
    executor, bit-exact vs MPICH's order on every rank."""
    P, n = 8, 64 << 20
    xs = [random_input(DT_FLOAT, n, 4242 + r) for r in range(P)]
    want = oracle.fold_ref_order(DT_FLOAT, xs)
    ins = [torch.from_numpy(x).to(gpu) for x in xs]
    outs = [torch.full_like(t, float('nan')) for t in ins]
    with config(lib, algo=algo, reference_order=1, tune=0, slice_bytes=2 << 20):
        _thread_allreduce(lib, ins, outs, n, DT_FLOAT)
    torch.cuda.synchronize()
    for r, o in enumerate(outs):
        assert o.cpu().numpy().tobytes() == want.tobytes(), r
    del ins, outs
    torch.cuda.empty_cache()


@pytest.mark.parametrize('P', [3, 8])
def test_thread_world_broadcast_allgatherv(lib, oracle, gpu, P):
    """RingExecutor::broadcast / allgatherv asynchronously (their programs have no reduce: the
    compute stream only forks and joins)."""
    s = torch.cuda.current_stream().cuda_stream
    with config(lib, slice_bytes=64 << 10):
        n, root = 300_007, P - 2
        xs = [random_input(DT_FLOAT, n, 900 + r) for r in range(P)]
        bufs = [torch.from_numpy(x).to(gpu) for x in xs]
        arr = (ctypes.c_void_p * P)(*[b.data_ptr() for b in bufs])
        assert lib.ddl_testing_thread_broadcast(P, root, arr, n, DT_FLOAT, s) == 0, lib.ddl_last_error()
        torch.cuda.synchronize()
        want = oracle.broadcast(DT_FLOAT, xs, root)
        for r in range(P):
            assert bufs[r].cpu().numpy().tobytes() == want[r].tobytes(), r
        counts = [10_000 * (r + 1) + 3 for r in range(P)]
        displs = list(np.cumsum([0] + counts[:-1]))
        xs = [random_input(DT_FLOAT, c, 950 + r) for r, c in enumerate(counts)]
        sends = [torch.from_numpy(x).to(gpu) for x in xs]
        recvs = [torch.full((sum(counts),), -1.0, device=gpu) for _ in range(P)]
        S = (ctypes.c_void_p * P)(*[t.data_ptr() for t in sends])
        R = (ctypes.c_void_p * P)(*[t.data_ptr() for t in recvs])
        C = (ctypes.c_size_t * P)(*counts)
        D = (ctypes.c_size_t * P)(*[int(d) for d in displs])
        assert lib.ddl_testing_thread_allgatherv(P, S, R, C, D, DT_FLOAT, s) == 0, lib.ddl_last_error()
        torch.cuda.synchronize()
        want = oracle.allgatherv(DT_FLOAT, xs)
        for r in range(P):
            assert recvs[r].cpu().numpy().tobytes() == want.tobytes(), r


def test_thread_world_repeated_calls_reuse_events(lib, oracle, gpu):
    """Back-to-back calls on the caller's stream with no host synchronisation in between (events,
    staging and the fabric's events reused): each result lands in its own output."""
    P, n = 5, 262_147
    with config(lib, algo=1, reference_order=1, tune=0, slice_bytes=64 << 10):
        cases = []
        for k in range(6):
            xs = [random_input(DT_FLOAT, n, 70 + 11 * k + r) for r in range(P)]
            ins = [torch.from_numpy(x).to(gpu) for x in xs]
            outs = [torch.empty_like(t) for t in ins]
            _thread_allreduce(lib, ins, outs, n, DT_FLOAT)
            cases.append((xs, outs))
        torch.cuda.synchronize()
        for xs, outs in cases:
            want = oracle.fold_ref_order(DT_FLOAT, xs).tobytes()
            assert all(o.cpu().numpy().tobytes() == want for o in outs)


def test_dropping_one_reduce_wait_is_caught(lib, oracle, gpu):
    """The mutation: RingExecutor skips the wait of the allgather tick on the fold it forwards
    (executor.cpp, tick.wait_reduce). Over the asynchronous transport the allgather's copies then
    read the output before the fold has written it, and the test sees wrong data; with the wait
    restored the same call is bit-exact again. (P = 8, one 32 MiB slice per chunk: the fold runs
    ~50 us, the copy starts at once.)"""
    P, n = 8, 64 << 20
    xs = [random_input(DT_FLOAT, n, 5150 + r) for r in range(P)]
    want = oracle.fold_ref_order(DT_FLOAT, xs).tobytes()
    ins = [torch.from_numpy(x).to(gpu) for x in xs]
    with config(lib, algo=1, reference_order=1, tune=0, slice_bytes=64 << 20):
        wrong = 0
        try:
            assert lib.ddl_testing_drop_wait(1) == 0  # tick 0 = reduce-scatter + fold, tick 1 = allgather
            for _ in range(3):
                outs = [torch.full_like(t, float('nan')) for t in ins]
                _thread_allreduce(lib, ins, outs, n, DT_FLOAT)
                torch.cuda.synchronize()
                wrong += sum(o.cpu().numpy().tobytes() != want for o in outs)
        finally:
            assert lib.ddl_testing_drop_wait(-1) == 0
        assert wrong > 0, 'dropping the allgather\'s wait on the fold went unnoticed'
        outs = [torch.full_like(t, float('nan')) for t in ins]
        _thread_allreduce(lib, ins, outs, n, DT_FLOAT)
        torch.cuda.synchronize()
        assert all(o.cpu().numpy().tobytes() == want for o in outs)
    del ins, outs
    torch.cuda.empty_cache()


@pytest.mark.parametrize('every,want', [(0, 256), (8, 224), (4, 192), (2, 128)])
def test_compute_stream_cu_mask(lib, gpu, every, want):
    """config compute_cu_mask: a multi-rank executor's compute stream (its reduce / fold kernels)
    leaves every n-th CU to RCCL — read back from the stream with hipExtStreamGetCUMask."""
    on, total = ctypes.c_int(), ctypes.c_int()
    assert lib.ddl_testing_compute_stream_cus(every, ctypes.byref(on), ctypes.byref(total)) == 0, lib.ddl_last_error()
    assert on.value == total.value * want // 256, (every, on.value, total.value)


@pytest.mark.parametrize('mask', [0, 2])
def test_masked_compute_stream_bit_exact(lib, oracle, gpu, mask):
    """The production executor with its compute stream masked (and unmasked; a thread world per
    mask): every rank still equals MPICH's order on a P = 8 direct allreduce whose chunks take the
    run-form fold."""
    P, n = 8, (9 << 20) // 4 * 8 + 5  # 9 MiB chunks: the run form at 8 inputs
    with config(lib, compute_cu_mask=mask, algo=1, reference_order=1, tune=0, slice_bytes=64 << 20):
        xs = [random_input(DT_FLOAT, n, 4242 + 7919 * r) for r in range(P)]
        ins = [_dev(x, gpu) for x in xs]
        outs = [torch.empty_like(t) for t in ins]
        _thread_allreduce(lib, ins, outs, n, DT_FLOAT)
        torch.cuda.synchronize()
        want = oracle.fold_ref_order(DT_FLOAT, xs).tobytes()
        for r in range(P):
            assert outs[r].cpu().numpy().tobytes() == want, r
