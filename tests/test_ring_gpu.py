"""The ring allreduce schedule on the GPU: P virtual ranks in one process, the exact per-rank
programs with HIP streams/events and the reduce kernel, device-to-device copies standing in for
RCCL send/recv (ddl_local_ring_allreduce). Checked against the oracle:
  * ring-order restatement: bit-exact for every dtype and P;
  * MPICH golden vectors: with reference_order (the default) bit-exact on every case; the ring
    order itself bit-exact where order-free (ints, P=2, exactly summable fp32), within the
    summation bound otherwise;
  * full-size (256 MiB fp32, C3 shape) through size-independent properties.
Tests of the ring / left-fold orders run with reference_order 0 (autouse fixture); the
reference-order tests opt back in.
"""
import ctypes
import json
import os

import numpy as np
import pytest
import torch

from _helpers import (ALL_DTYPES, DT_FLOAT, DT_HALF, FROM_NP, NAME, config, fp16_single_rounding_bound, random_input, ring_perms,
                      ring_shape)

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.fixture(autouse=True)
def _schedules_as_configured(lib):
    with config(lib, reference_order=0):
        yield


def run_local(lib, dev, xs, in_place=False, stream=None):
    ins = [torch.from_numpy(np.ascontiguousarray(x)).to(dev) for x in xs]
    outs = ins if in_place else [torch.empty_like(t) for t in ins]
    P = len(xs)
    send = (ctypes.c_void_p * P)(*[t.data_ptr() for t in ins])
    recv = (ctypes.c_void_p * P)(*[t.data_ptr() for t in outs])
    dt = FROM_NP.get(str(xs[0].dtype), 14)
    s = torch.cuda.current_stream().cuda_stream if stream is None else stream
    st = lib.ddl_local_ring_allreduce(P, send, recv, xs[0].size, dt, 0, s)
    assert st == 0, lib.ddl_last_error()
    torch.cuda.synchronize()
    return [o.cpu().numpy().view(xs[0].dtype) for o in outs]


@pytest.mark.parametrize('P', [1, 2, 3, 4, 5, 8])
@pytest.mark.parametrize('dt', [d for d in ALL_DTYPES if d != 14], ids=lambda d: NAME[d])  # bf16: below
@pytest.mark.parametrize('n', [1, 257, 65_537, 1_000_003])
def test_local_ring_matches_ring_oracle(lib, oracle, gpu, P, dt, n):
    xs = [random_input(dt, n, 1234 + 7919 * r) for r in range(P)]
    outs = run_local(lib, gpu, xs)
    R, _ = ring_shape(lib, n, dt, P)
    want = oracle.allreduce_ring(dt, xs, ring_perms(lib, P, R))
    for r in range(P):
        assert outs[r].tobytes() == want.tobytes(), f'rank {r}'


def test_local_ring_bf16(lib, oracle, gpu):
    P, n, dt = 8, 300_007, 14
    xs = [random_input(dt, n, 1234 + 7919 * r) for r in range(P)]
    ins = [torch.from_numpy(x.view(np.int16)).to(gpu) for x in xs]
    outs = [torch.empty_like(t) for t in ins]
    send = (ctypes.c_void_p * P)(*[t.data_ptr() for t in ins])
    recv = (ctypes.c_void_p * P)(*[t.data_ptr() for t in outs])
    assert lib.ddl_local_ring_allreduce(P, send, recv, n, dt, 0, torch.cuda.current_stream().cuda_stream) == 0
    torch.cuda.synchronize()
    R, _ = ring_shape(lib, n, dt, P)
    want = oracle.allreduce_ring(dt, xs, ring_perms(lib, P, R))
    for o in outs:
        assert o.cpu().numpy().view(np.uint16).tobytes() == want.tobytes()


@pytest.mark.parametrize('P', [2, 8])
def test_local_ring_in_place(lib, oracle, gpu, P):
    n = 1 << 20
    xs = [random_input(DT_FLOAT, n, 99 + r) for r in range(P)]
    outs = run_local(lib, gpu, xs, in_place=True)
    R, _ = ring_shape(lib, n, DT_FLOAT, P)
    want = oracle.allreduce_ring(DT_FLOAT, xs, ring_perms(lib, P, R))
    for o in outs:
        assert o.tobytes() == want.tobytes()


def _golden():
    gold = np.load(os.path.join(HERE, 'golden', 'golden_mpich.npz'), allow_pickle=False)
    meta = json.load(open(os.path.join(HERE, 'golden', 'golden_manifest.json')))['cases']
    return [(case, m, gold[case + '__inputs'], gold[case + '__output']) for case, m in meta.items()]


def test_local_ring_vs_mpich_golden(lib, gpu):
    """Ring order (reference_order 0) against MPICH's outputs: exact where order-free, else
    within the bound between two summation orders, 2 (P-1) u sum|x|."""
    for case, m, xs, y in _golden():
        outs = run_local(lib, gpu, list(xs))
        exact = np.issubdtype(xs.dtype, np.integer) or m['P'] == 2 or m['kind'] != 'randn'
        for o in outs:
            if exact:
                assert o.tobytes() == y.tobytes(), case
            else:
                u = np.finfo(xs.dtype).eps / 2
                bound = 2 * (m['P'] - 1) * u * np.abs(xs.astype(np.float64)).sum(0) * 1.0001
                assert np.all(np.abs(o.astype(np.float64) - y.astype(np.float64)) <= bound), case


@pytest.mark.parametrize('algo', [0, 1, 2, 3])
def test_reference_order_equals_mpich_golden_bit_for_bit(lib, gpu, algo):
    """The product default (reference_order 1): every golden case — MPICH 3.3.2's own
    MPI_Allreduce outputs at P = 2..8, fp32 / fp64 / integers, both sides of its 2048-byte
    algorithm switch — comes out of the GPU bit for bit on every rank, whichever schedule is
    asked for (a ring at P > 2 runs as the direct schedule; one-shot beyond its tuning range
    still works)."""
    with config(lib, algo=algo, reference_order=1, slice_bytes=64 << 10):
        for case, m, xs, y in _golden():
            for o in run_local(lib, gpu, list(xs)):
                assert o.tobytes() == y.tobytes(), case


@pytest.mark.parametrize('algo', [1, 2, 3, 4])
@pytest.mark.parametrize('P', [3, 5, 6, 7, 8])
@pytest.mark.parametrize('dt', [1, 2, 3], ids=lambda d: NAME[d])
@pytest.mark.parametrize('n', [1, 300, 512, 513, 65_537, 1_000_003, 128 * 840])
@pytest.mark.parametrize('in_place', [False, True])
def test_reference_order_matches_oracle(lib, oracle, gpu, algo, P, dt, n, in_place):
    """The ordered fold kernels (binomial, pre-fold + pairwise tree) through the direct and
    one-shot programs vs the oracle's MPICH-order restatement, in and out of place, ragged
    (128 * 840 elements: equal chunks at every P here, so direct-gather's collective allgather)."""
    xs = [random_input(dt, n, 61 + 5 * r) for r in range(P)]
    with config(lib, algo=algo, reference_order=1, slice_bytes=256 << 10):
        outs = run_local(lib, gpu, xs, in_place=in_place)
    want = oracle.fold_ref_order(dt, xs)
    for r in range(P):
        assert outs[r].tobytes() == want.tobytes(), f'rank {r}'


def test_reference_order_misaligned_fold(lib, oracle, gpu):
    """The element-granular ordered fold (inputs not 16-byte aligned) at P = 5, both orders."""
    P = 5
    for n in (301, 100_003):
        xs = [random_input(1, n + 1, 3 + r) for r in range(P)]
        ins = [torch.from_numpy(x).to(gpu)[1:] for x in xs]
        outs = [torch.empty(n + 1, dtype=torch.float32, device=gpu)[1:] for _ in range(P)]
        send = (ctypes.c_void_p * P)(*[t.data_ptr() for t in ins])
        recv = (ctypes.c_void_p * P)(*[t.data_ptr() for t in outs])
        with config(lib, algo=1, reference_order=1):
            assert lib.ddl_local_ring_allreduce(P, send, recv, n, 1, 0, torch.cuda.current_stream().cuda_stream) == 0
            torch.cuda.synchronize()
        want = oracle.fold_ref_order(1, [x[1:] for x in xs])
        for o in outs:
            assert o.cpu().numpy().tobytes() == want.tobytes(), n


@pytest.mark.parametrize('P', [4, 8])
def test_reference_order_tuner_times_only_exact_schedules(lib, gpu, P):
    """With reference_order the autotuner's candidates are direct / one-shot / gather-fold /
    direct-gather schedules only at P > 2 (the configured ring becomes direct), deduplicated;
    direct-gather only where the chunks are equal (64 KiB at P = 4, 8: yes; 64 KiB + 256 B: no)."""
    chosen, count = ctypes.c_int(), ctypes.c_int()
    cfgs = (ctypes.c_longlong * 64)()
    ms = (ctypes.c_float * 16)()
    with config(lib, reference_order=1, algo=0):
        st = lib.ddl_local_tune(P, 64 << 10, DT_FLOAT, torch.cuda.current_stream().cuda_stream,
                                ctypes.byref(chosen), ctypes.byref(count), cfgs, ms, 16)
    assert st == 0, lib.ddl_last_error()
    c = [tuple(cfgs[4 * i:4 * i + 4]) for i in range(count.value)]
    assert {x[0] for x in c} == {1, 2, 3, 4} and len(set(c)) == len(c)
    assert c[0][0] == 1
    with config(lib, reference_order=1, algo=0):
        st = lib.ddl_local_tune(P, (64 << 10) + 64, DT_FLOAT, torch.cuda.current_stream().cuda_stream,
                                ctypes.byref(chosen), ctypes.byref(count), cfgs, ms, 16)
    assert st == 0, lib.ddl_last_error()
    assert {cfgs[4 * i] for i in range(count.value)} == {1, 2, 3}


@pytest.mark.parametrize('P', [2, 4, 8])
def test_reference_known_answer(lib, gpu, P):
    """allreduce_test.py:13: fp32[16] filled with rank -> P(P-1)/2 on every rank."""
    xs = [np.full(16, r, np.float32) for r in range(P)]
    for o in run_local(lib, gpu, xs):
        assert np.all(o == P * (P - 1) / 2)


def test_full_size_256mib_properties(lib, gpu):
    """C3 shape: one 256 MiB fp32 bucket per rank at P=8. Exactly summable inputs make the
    sum order-free, so every rank must equal the rank-order sum computed by torch in fp64
    (exact) — a size-independent check at full size."""
    P, n = 8, 64 << 20
    g = torch.Generator(device=gpu).manual_seed(5)
    ins = [(torch.randint(-(2 ** 12) + 1, 2 ** 12, (n,), device=gpu, generator=g).float() * 2.0 ** -10)
           for _ in range(P)]
    want = torch.stack(ins).double().sum(0).float()
    outs = [torch.empty_like(t) for t in ins]
    send = (ctypes.c_void_p * P)(*[t.data_ptr() for t in ins])
    recv = (ctypes.c_void_p * P)(*[t.data_ptr() for t in outs])
    assert lib.ddl_local_ring_allreduce(P, send, recv, n, DT_FLOAT, 0, torch.cuda.current_stream().cuda_stream) == 0
    torch.cuda.synchronize()
    for o in outs:
        assert torch.equal(o, want)


def test_fp16_tolerance_vs_fp64(lib, oracle, gpu):
    """fp16 (no reference oracle: the reference rejects it). Reference order at P = 8 runs the
    direct schedule: all inputs folded in fp32, ONE rounding, so
    |y - sum64| <= ulp16(y)/2 + (P-1) * 2^-24 * sum|x|, and y equals the oracle's fp16 rule bit for
    bit. reference_order 0 (a ring, rounding at every hop) keeps the per-hop bound
    (P-1) * 2^-11 * sum|x| + ulp16/2."""
    P, n = 8, 1 << 20
    xs = [random_input(DT_HALF, n, 500 + r) for r in range(P)]
    exact = np.sum([x.astype(np.float64) for x in xs], axis=0)
    mag = np.sum([np.abs(x.astype(np.float64)) for x in xs], axis=0)
    with config(lib, reference_order=1):
        y = run_local(lib, gpu, xs)[0]
    assert y.tobytes() == oracle.fold_ref_order(DT_HALF, xs).tobytes()
    bound = fp16_single_rounding_bound(P, torch.from_numpy(y), torch.from_numpy(mag)).numpy()
    assert np.all(np.abs(y.astype(np.float64) - exact) <= bound)
    with config(lib, reference_order=0):
        out = run_local(lib, gpu, xs)[0].astype(np.float64)
    ulp = np.spacing(np.abs(exact).astype(np.float16)).astype(np.float64)
    assert np.all(np.abs(out - exact) <= (P - 1) * 2.0 ** -11 * mag + ulp / 2)


def test_repeated_calls_reuse_resources(lib, oracle, gpu):
    """Events/staging are reused across calls and across sizes (growth path)."""
    for n in (1000, 5_000_000, 3000, 8_000_000):
        xs = [random_input(DT_FLOAT, n, 7 + r) for r in range(4)]
        outs = run_local(lib, gpu, xs)
        R, _ = ring_shape(lib, n, DT_FLOAT, 4)
        want = oracle.allreduce_ring(DT_FLOAT, xs, ring_perms(lib, 4, R))
        assert all(o.tobytes() == want.tobytes() for o in outs)


# ---- direct (all-to-all) schedule: algo = 1 ------------------------------------------------
@pytest.mark.parametrize('P', [2, 3, 4, 5, 8])
@pytest.mark.parametrize('dt', ALL_DTYPES, ids=lambda d: NAME[d])
@pytest.mark.parametrize('n', [1, 257, 65_537, 1_000_003])
def test_local_direct_matches_direct_oracle(lib, oracle, gpu, P, dt, n):
    """The N-input fold kernel (fp32 accumulation for fp16/bf16, one rounding) over the direct
    schedule's per-rank programs, bit-exact vs the oracle's direct fold."""
    xs = [random_input(dt, n, 4321 + 17 * r) for r in range(P)]
    with config(lib, algo=1):
        if dt == 14:
            ins = [torch.from_numpy(x.view(np.int16)).to(gpu) for x in xs]
            outs = [torch.empty_like(t) for t in ins]
            send = (ctypes.c_void_p * P)(*[t.data_ptr() for t in ins])
            recv = (ctypes.c_void_p * P)(*[t.data_ptr() for t in outs])
            st = lib.ddl_local_ring_allreduce(P, send, recv, n, dt, 0, torch.cuda.current_stream().cuda_stream)
            assert st == 0, lib.ddl_last_error()
            torch.cuda.synchronize()
            outs = [o.cpu().numpy().view(np.uint16) for o in outs]
        else:
            outs = run_local(lib, gpu, xs)
    want = oracle.allreduce_direct(dt, xs)
    for r in range(P):
        assert outs[r].tobytes() == want.tobytes(), f'rank {r}'


@pytest.mark.parametrize('P', [2, 8])
def test_local_direct_in_place_and_slices(lib, oracle, gpu, P):
    n = (3 << 20) + 5  # several slices per chunk at 64 KiB slices, ragged tail
    xs = [random_input(DT_FLOAT, n, 77 + r) for r in range(P)]
    with config(lib, algo=1, slice_bytes=64 << 10):
        outs = run_local(lib, gpu, xs, in_place=True)
    want = oracle.allreduce_direct(DT_FLOAT, xs)
    for o in outs:
        assert o.tobytes() == want.tobytes()


def test_local_direct_full_size_256mib(lib, gpu):
    """C3 shape (256 MiB fp32, P=8) through the direct schedule: exactly summable inputs, every
    rank equals the fp64 sum."""
    P, n = 8, 64 << 20
    g = torch.Generator(device=gpu).manual_seed(6)
    ins = [(torch.randint(-(2 ** 12) + 1, 2 ** 12, (n,), device=gpu, generator=g).float() * 2.0 ** -10)
           for _ in range(P)]
    want = torch.stack(ins).double().sum(0).float()
    outs = [torch.empty_like(t) for t in ins]
    send = (ctypes.c_void_p * P)(*[t.data_ptr() for t in ins])
    recv = (ctypes.c_void_p * P)(*[t.data_ptr() for t in outs])
    with config(lib, algo=1):
        assert lib.ddl_local_ring_allreduce(P, send, recv, n, DT_FLOAT, 0,
                                            torch.cuda.current_stream().cuda_stream) == 0
        torch.cuda.synchronize()
    for o in outs:
        assert torch.equal(o, want)


def test_reduce_sumN_kernel_all_input_counts(lib, oracle, gpu):
    """The N-input fold kernel alone for every supported input count (1..15 received inputs),
    aligned and misaligned, through a P-rank direct run with P = nb + 1 up to 16 ranks."""
    for P in (9, 12, 16):
        n = 10_001
        xs = [random_input(DT_HALF, n, 5 + r) for r in range(P)]
        with config(lib, algo=1):
            outs = run_local(lib, gpu, xs)
        want = oracle.allreduce_direct(DT_HALF, xs)
        assert outs[0].tobytes() == want.tobytes(), P


@pytest.mark.parametrize('P,ncand', [(2, 4), (4, 13), (8, 13)])
def test_local_autotune_candidates(lib, gpu, P, ncand):
    """The autotuner's procedure on P virtual ranks: the configured schedule is candidate 0,
    every candidate is timed, the chosen one is the fastest (4 MiB: equal chunks at P = 4, 8, so
    the direct-gather candidates too; chunks <= 4 MiB, so direct with 256 KiB slices too)."""
    chosen, count = ctypes.c_int(), ctypes.c_int()
    cfgs = (ctypes.c_longlong * 64)()
    ms = (ctypes.c_float * 16)()
    st = lib.ddl_local_tune(P, 4 << 20, DT_FLOAT, torch.cuda.current_stream().cuda_stream,
                            ctypes.byref(chosen), ctypes.byref(count), cfgs, ms, 16)
    assert st == 0, lib.ddl_last_error()
    assert count.value == ncand
    assert (cfgs[0], cfgs[1], cfgs[2]) == (lib.ddl_get_config(b'algo'), lib.ddl_get_config(b'rings'),
                                           lib.ddl_get_config(b'slice_bytes'))
    times = [ms[i] for i in range(count.value)]
    assert all(t > 0 for t in times)
    assert times[chosen.value] == min(times)
    algos = {cfgs[4 * i] for i in range(count.value)}
    assert algos == ({0, 1, 4} if P > 2 else {0})
    if P > 2:
        assert (1, 256 << 10) in {(cfgs[4 * i], cfgs[4 * i + 2]) for i in range(count.value)}


# ---- one-shot schedule: algo = 2 --------------------------------------------------------------
@pytest.mark.parametrize('P', [2, 3, 5, 8])
@pytest.mark.parametrize('dt', [d for d in ALL_DTYPES if d != 14], ids=lambda d: NAME[d])
@pytest.mark.parametrize('n', [1, 257, 65_537, 300_001])
@pytest.mark.parametrize('in_place', [False, True])
def test_local_oneshot_matches_rank_order_fold(lib, oracle, gpu, P, dt, n, in_place):
    """One group of whole-bucket exchanges, then the N-input fold in rank order on every rank:
    every rank equals the oracle's rank-order fold bit for bit, in and out of place."""
    xs = [random_input(dt, n, 97 + 3 * r) for r in range(P)]
    with config(lib, algo=2):
        outs = run_local(lib, gpu, xs, in_place=in_place)
    want = oracle.fold(dt, xs)
    for r in range(P):
        assert outs[r].tobytes() == want.tobytes(), f'rank {r}'


def test_local_oneshot_repeated_calls(lib, oracle, gpu):
    """Back-to-back one-shot calls reuse staging: the next call's receives must not land while
    the previous call's fold still reads (the caller joins on the fold)."""
    P, n = 8, 1 << 18
    with config(lib, algo=2):
        for it in range(6):
            xs = [random_input(DT_FLOAT, n, 1000 * it + r) for r in range(P)]
            outs = run_local(lib, gpu, xs)
            want = oracle.fold(DT_FLOAT, xs)
            assert all(o.tobytes() == want.tobytes() for o in outs), it


def test_local_autotune_small_bucket_tries_oneshot(lib, gpu):
    chosen, count = ctypes.c_int(), ctypes.c_int()
    cfgs = (ctypes.c_longlong * 64)()
    ms = (ctypes.c_float * 16)()
    st = lib.ddl_local_tune(8, 64 << 10, DT_FLOAT, torch.cuda.current_stream().cuda_stream,
                            ctypes.byref(chosen), ctypes.byref(count), cfgs, ms, 16)
    assert st == 0, lib.ddl_last_error()
    assert 2 in {cfgs[4 * i] for i in range(count.value)}
    times = [ms[i] for i in range(count.value)]
    assert times[chosen.value] == min(times)


@pytest.mark.parametrize('algo', [0, 1])
def test_bucket_beyond_2pow31_elements(lib, gpu, algo):
    """Maximum-size bucket: 2^31 + 4099 fp16 elements per rank (4 GiB; the reference's
    MPI_Allreduce takes `(int) elements` and cannot express it, MPICommunicator.cc:19). Two
    virtual ranks, exactly summable inputs, so every element must equal the torch sum; checks
    64-bit indexing in the partition, the tick programs and the kernels."""
    P, n = 2, (1 << 31) + 4099
    base = (torch.arange(n, device=gpu, dtype=torch.int32) % 7).half()
    ins = [base + float(r) for r in range(P)]
    want = base * P + float(sum(range(P)))
    send = (ctypes.c_void_p * P)(*[t.data_ptr() for t in ins])
    with config(lib, algo=algo):
        assert lib.ddl_local_ring_allreduce(P, send, send, n, DT_HALF, 0, torch.cuda.current_stream().cuda_stream) == 0
        torch.cuda.synchronize()
    for t in ins:
        assert torch.equal(t, want)
    del ins, base, want
    torch.cuda.empty_cache()


def test_random_configurations_on_gpu(lib, oracle, gpu):
    """Random (P, n, dtype, algo, reference_order, slicing, rings, in place) through the real
    streams and kernels on virtual ranks: every rank holds the sum the configuration promises,
    bit for bit (MPICH's order with reference_order; ring / left-fold / rank-order otherwise)."""
    rng = np.random.default_rng(77)
    for trial in range(40):
        P = int(rng.integers(2, 9))
        n = int(rng.choice([1, 65, 511, 513, 4099, 100_003, 1_000_003]))
        dt = int(rng.choice([d for d in ALL_DTYPES if d != 14]))
        algo, ref = int(rng.integers(0, 3)), int(rng.integers(0, 2))
        kv = dict(algo=algo, reference_order=ref, slice_bytes=int(rng.choice([4 << 10, 256 << 10, 2 << 20])),
                  max_slices=int(rng.integers(1, 17)), rings=int(rng.integers(1, 9)))
        xs = [random_input(dt, n, 5 * trial + r) for r in range(P)]
        with config(lib, **kv):
            outs = run_local(lib, gpu, xs, in_place=bool(trial % 2))
            R, _ = ring_shape(lib, n, dt, P)
            perms = ring_perms(lib, P, R, max_rings=kv['rings'])
        if ref and (algo != 0 or P > 2):
            want = oracle.fold_ref_order(dt, xs)
        elif algo == 0:
            want = oracle.allreduce_ring(dt, xs, perms)
        elif algo == 1:
            want = oracle.allreduce_direct(dt, xs)
        else:
            want = oracle.fold(dt, xs)
        for r in range(P):
            assert outs[r].tobytes() == want.tobytes(), (trial, P, n, dt, kv, r)


@pytest.mark.parametrize('P', [17, 33])
@pytest.mark.parametrize('algo,ref', [(0, 1), (1, 1), (2, 1), (1, 0), (2, 0)])
@pytest.mark.parametrize('dt', [1, 2, 3], ids=lambda d: NAME[d])
def test_fold_trees_beyond_sixteen_ranks_on_gpu(lib, oracle, gpu, P, algo, ref, dt):
    """Beyond 16 virtual ranks the fold runs as several launches through staging partials (a
    left chain, or MPICH's tree in blocks of 16): bit-exact with the requested order, in place,
    on both sides of the 2048-byte switch."""
    for n in (300, 100_003):
        xs = [random_input(dt, n, 7 * P + 3 * r + n) for r in range(P)]
        with config(lib, algo=algo, reference_order=ref, slice_bytes=64 << 10):
            outs = run_local(lib, gpu, xs, in_place=True)
        if ref:
            want = oracle.fold_ref_order(dt, xs)
        else:
            want = oracle.allreduce_direct(dt, xs) if algo == 1 else oracle.fold(dt, xs)
        for r in range(P):
            assert outs[r].tobytes() == want.tobytes(), (n, r)


def test_reference_order_mpich_golden_beyond_8_ranks(lib, gpu):
    """MPICH's own outputs at P = 17, 20, 33 (one host, tests/golden/golden_mpich_bigp.npz) from
    the GPU's virtual ranks bit for bit: fold trees of more than 16 inputs through staging
    partials, every schedule."""
    gold = np.load(os.path.join(HERE, 'golden', 'golden_mpich_bigp.npz'), allow_pickle=False)
    meta = json.load(open(os.path.join(HERE, 'golden', 'golden_manifest_bigp.json')))['cases']
    for algo in (0, 1, 2, 3):
        with config(lib, algo=algo, reference_order=1, slice_bytes=64 << 10):
            for case, m in sorted(meta.items()):
                if m['P'] > 64:
                    continue
                for o in run_local(lib, gpu, list(gold[case + '__inputs'])):
                    assert o.tobytes() == gold[case + '__output'].tobytes(), (algo, case)
