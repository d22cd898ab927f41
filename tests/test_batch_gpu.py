"""The grouped allreduce (ddl_allreduce_batch; RingExecutor::allreduce_batch): `count` buckets of
one dtype as ONE program — per tick one group with every bucket's slices, the folds of up to 8
buckets per launch (FoldBatch, blockIdx.y = bucket). Bar: every bucket bit for bit what the
per-bucket allreduce gives it (MPICH's order for its own message size: ddlo_fold_ref_order), on
every rank, through

  * the production executor driven asynchronously (the thread world),
  * the RCCL transport (one-rank loopback: every matched pair through RCCL, hundreds per group),
  * the batched fold kernel alone (ddl_reduce_fold_batch) vs the oracle;

and the posted dependencies race-free (deptrace.h). Reference semantics: each bucket is its own
MPI_Allreduce (MPICommunicator.cc:14-28)."""
import ctypes

import numpy as np
import pytest
import torch

from _helpers import DT_DOUBLE, DT_FLOAT, DT_HALF, DT_INT32, NAME, config, random_input

pytestmark = pytest.mark.gpu
VP, SZ = ctypes.c_void_p, ctypes.c_size_t


def _dev(x, gpu):
    if x.dtype == np.float16:
        return torch.from_numpy(x.view(np.int16)).to(gpu).view(torch.float16)
    return torch.from_numpy(np.ascontiguousarray(x)).to(gpu)


def _host(t, like):
    if like.dtype == np.float16:
        return t.view(torch.int16).cpu().numpy().view(np.float16)
    return t.cpu().numpy()


def _batch(fn, P, ins, outs, ns, dt):
    k = len(ns)
    S = (VP * (P * k))(*[ins[r][b].data_ptr() for r in range(P) for b in range(k)])
    D = (VP * (P * k))(*[outs[r][b].data_ptr() for r in range(P) for b in range(k)])
    return fn(P, k, S, D, (SZ * k)(*ns), dt, torch.cuda.current_stream().cuda_stream)


SIZES = [1, 300, 0, 65_537, 257, 1_000_003, 128 * 840, 5, 2 << 20, 513]  # ragged, empty, both sides of 2048 B


@pytest.mark.parametrize('P', [2, 3, 5, 8])
@pytest.mark.parametrize('algo', [1, 2, 4])
@pytest.mark.parametrize('dt', [DT_FLOAT, DT_DOUBLE, DT_INT32, DT_HALF], ids=lambda d: NAME[d])
def test_thread_batch_bit_exact_per_bucket(lib, oracle, gpu, P, algo, dt):
    """10 buckets (empty, 1 element, ragged, 8 MiB) through the production executor as one grouped
    program; every bucket equals MPICH's order for its own message on every rank. algo 4
    (direct-gather) runs as direct inside a batch; 64 KiB slices: several ticks per bucket, the
    buckets' tick counts differ."""
    ns = SIZES if dt != DT_HALF else [n for n in SIZES if n != 1_000_003]
    xs = [[random_input(dt, n, 7000 * r + 31 * b + P) for b, n in enumerate(ns)] for r in range(P)]
    ins = [[_dev(x, gpu) for x in row] for row in xs]
    in_place = algo == 2
    outs = ins if in_place else [[torch.full_like(t, 0) for t in row] for row in ins]
    with config(lib, algo=algo, reference_order=1, tune=0, slice_bytes=64 << 10):
        st = _batch(lib.ddl_testing_thread_allreduce_batch, P, ins, outs, ns, dt)
        assert st == 0, lib.ddl_last_error()
        torch.cuda.synchronize()
    for b, n in enumerate(ns):
        if n == 0:
            continue
        want = oracle.fold_ref_order(dt, [xs[r][b] for r in range(P)]).tobytes()
        for r in range(P):
            assert _host(outs[r][b], xs[r][b]).tobytes() == want, (b, n, r)


@pytest.mark.parametrize('algo', [0, 1, 2])
@pytest.mark.parametrize('dt', [DT_FLOAT, DT_DOUBLE], ids=lambda d: NAME[d])
def test_thread_batch_reference_order_0(lib, oracle, gpu, algo, dt):
    """with reference_order 0 the grouped allreduce sums every bucket in the
    batch schedule's order — the direct rank-order fold, or the one-shot left fold where one-shot
    is asked for (a ring request runs as direct inside a batch) — as include/ddl_amd.h now states;
    a solo call of a ring-tuned size class may differ in the last bits, so the claim of equality
    with ddl_allreduce is made for reference_order 1 only (test above)."""
    P = 5
    ns = [300, 65_537, 1_000_003, 5]
    xs = [[random_input(dt, n, 900 * r + 7 * b + algo) for b, n in enumerate(ns)] for r in range(P)]
    ins = [[_dev(x, gpu) for x in row] for row in xs]
    outs = [[torch.full_like(t, 0) for t in row] for row in ins]
    with config(lib, algo=algo, reference_order=0, tune=0, slice_bytes=64 << 10):
        st = _batch(lib.ddl_testing_thread_allreduce_batch, P, ins, outs, ns, dt)
        assert st == 0, lib.ddl_last_error()
        torch.cuda.synchronize()
    for b, n in enumerate(ns):
        col = [xs[r][b] for r in range(P)]
        want = (oracle.fold(dt, col) if algo == 2 else oracle.allreduce_direct(dt, col)).tobytes()
        for r in range(P):
            assert _host(outs[r][b], xs[r][b]).tobytes() == want, (algo, b, n, r)


@pytest.mark.parametrize('P', [3, 8])
def test_rccl_loopback_batch(lib, oracle, gpu, P):
    """The same grouped program with every matched pair through RCCL (one-rank loopback): a tick's
    group carries the pairs of every bucket of every virtual rank."""
    assert lib.ddl_rccl_loopback_init(0) == 0, lib.ddl_last_error()
    try:
        ns = SIZES
        xs = [[random_input(DT_FLOAT, n, 900 * r + b) for b, n in enumerate(ns)] for r in range(P)]
        ins = [[_dev(x, gpu) for x in row] for row in xs]
        outs = [[torch.empty_like(t) for t in row] for row in ins]
        with config(lib, algo=1, reference_order=1, tune=0, slice_bytes=256 << 10):
            assert _batch(lib.ddl_rccl_loopback_allreduce_batch, P, ins, outs, ns, DT_FLOAT) == 0, lib.ddl_last_error()
            torch.cuda.synchronize()
        for b, n in enumerate(ns):
            if n:
                want = oracle.fold_ref_order(DT_FLOAT, [xs[r][b] for r in range(P)]).tobytes()
                for r in range(P):
                    assert outs[r][b].cpu().numpy().tobytes() == want, (b, r)
    finally:
        assert lib.ddl_rccl_loopback_finalize() == 0, lib.ddl_last_error()


def test_local_batch_equals_per_bucket_p17(lib, oracle, gpu):
    """P = 17 (folds split beyond 16 inputs: chained steps through partials, which may not share a
    launch) through the one-GPU copy world: bit-exact vs MPICH's order per bucket."""
    P = 17
    ns = [300, 65_537, 4096, 0, 100_003]
    xs = [[random_input(DT_FLOAT, n, 50 * r + b) for b, n in enumerate(ns)] for r in range(P)]
    ins = [[_dev(x, gpu) for x in row] for row in xs]
    outs = [[torch.empty_like(t) for t in row] for row in ins]
    with config(lib, algo=1, reference_order=1, tune=0, slice_bytes=64 << 10):
        assert _batch(lib.ddl_local_allreduce_batch, P, ins, outs, ns, DT_FLOAT) == 0, lib.ddl_last_error()
        torch.cuda.synchronize()
    for b, n in enumerate(ns):
        if n:
            want = oracle.fold_ref_order(DT_FLOAT, [xs[r][b] for r in range(P)]).tobytes()
            for r in range(P):
                assert outs[r][b].cpu().numpy().tobytes() == want, (b, r)


def test_c4_as_one_batch_equals_per_bucket(lib, gpu):
    """C4 (64 x 16 MiB fp16 per rank, P = 8) as ONE grouped call through the production executor:
    every bucket bit-identical to the same bucket reduced alone (ddl_testing_thread_allreduce), so
    the batch inherits C4's fp16 bound and its oracle check (test_thread_world_gpu.py)."""
    P, nb, k = 8, (16 << 20) // 2, 64
    g = torch.Generator(device=gpu).manual_seed(404)
    ins = [[(torch.randn(nb, device=gpu, generator=g) * 0.1).half() for _ in range(k)] for _ in range(P)]
    outs = [[torch.empty_like(t) for t in row] for row in ins]
    s = torch.cuda.current_stream().cuda_stream
    with config(lib, algo=1, reference_order=1, tune=0, slice_bytes=2 << 20):
        assert _batch(lib.ddl_testing_thread_allreduce_batch, P, ins, outs, [nb] * k, DT_HALF) == 0, \
            lib.ddl_last_error()
        ref = [torch.empty_like(t) for t in ins[0]]
        for b in range(0, k, 9):  # every 9th bucket alone, rank by rank outputs compared
            single = [torch.empty_like(ins[0][b]) for _ in range(P)]
            S = (VP * P)(*[ins[r][b].data_ptr() for r in range(P)])
            D = (VP * P)(*[t.data_ptr() for t in single])
            assert lib.ddl_testing_thread_allreduce(P, S, D, nb, DT_HALF, s) == 0, lib.ddl_last_error()
            ref[b] = single
        torch.cuda.synchronize()
    for b in range(0, k, 9):
        for r in range(P):
            assert torch.equal(outs[r][b], ref[b][r]), (b, r)
    del ins, outs, ref
    torch.cuda.empty_cache()


@pytest.mark.parametrize('P', [3, 8])
def test_batch_posted_dependencies_have_no_race(lib, gpu, P):
    """What a grouped call posts — merged ticks, batched folds, the merged wait on the latest
    reduce — orders every conflicting pair (deptrace.h), in place, mixed slice counts."""
    ns = [300, 0, 65_537, 128 * 840 + 3, 2 << 20, 17]
    ins = [[torch.randn(n, device=gpu) for n in ns] for _ in range(P)]
    torch.cuda.synchronize()
    with config(lib, algo=1, reference_order=1, tune=0, slice_bytes=64 << 10):
        assert lib.ddl_testing_dep_trace(1) == 0
        try:
            assert _batch(lib.ddl_testing_thread_allreduce_batch, P, ins, ins, ns, DT_FLOAT) == 0, lib.ddl_last_error()
        finally:
            assert lib.ddl_testing_dep_trace(0) == 0
        torch.cuda.synchronize()
    counts = (ctypes.c_longlong * 5)()
    buf = ctypes.create_string_buffer(1 << 14)
    assert lib.ddl_testing_dep_check(counts, buf, len(buf)) == 0
    assert counts[4] == 0, buf.value.decode()
    assert counts[3] > 0, list(counts)


@pytest.mark.parametrize('dt', [DT_FLOAT, DT_HALF, DT_DOUBLE], ids=lambda d: NAME[d])
@pytest.mark.parametrize('order', [0, 1])
def test_fold_batch_kernel_vs_oracle(lib, oracle, gpu, dt, order):
    """ddl_reduce_fold_batch: 8 problems of different lengths (ragged tails) in one launch, each
    bit-exact vs the oracle's fold of its own inputs (fp16: rank order in fp32, one rounding)."""
    nb, ns = 7, [1, 4096 + 3, 300, 1 << 20, 65_537, 0, 2 * 1024 * 1024 // 2 + 5, 1024]
    k = len(ns)
    xs = [[random_input(dt, n, 300 * p + i) for i in range(nb + 1)] for p, n in enumerate(ns)]
    dev = [[_dev(x, gpu) for x in row] for row in xs]
    outs = [torch.empty_like(row[0]) for row in dev]
    A = (VP * k)(*[row[0].data_ptr() for row in dev])
    B = (VP * (k * nb))(*[t.data_ptr() for row in dev for t in row[1:]])
    O = (VP * k)(*[t.data_ptr() for t in outs])
    s = torch.cuda.current_stream().cuda_stream
    assert lib.ddl_reduce_fold_batch(k, O, A, B, nb, (SZ * k)(*ns), dt, order if dt != DT_HALF else 0, s) == 0, \
        lib.ddl_last_error()
    torch.cuda.synchronize()
    for p, n in enumerate(ns):
        if n == 0:
            continue
        if order == 1 and dt != DT_HALF:
            want = oracle.fold_ref_order(dt, xs[p], 1 << 30)
        else:
            want = oracle.fold(dt, xs[p])
        assert _host(outs[p], xs[p][0]).tobytes() == want.tobytes(), (p, n)
