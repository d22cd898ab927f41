"""Pin the oracle (oracle/ddl_oracle.c) against the golden vectors before trusting it.

Golden vectors (tests/golden/make_golden.py): MPICH 3.3.2 MPI_Allreduce(MPI_SUM) — the
reference's data-plane call, src/cpp/communicate/backend/mpi/MPICommunicator.cc:14-28 — run
with mpiexec -n P; the reference's own known answer (src/py/ddl/test/allreduce_test.py:13);
and the reference outputs recorded in SURVEY.md §4.

Parity bar: the oracle's restatement of MPICH's own summation order (ddlo_fold_ref_order:
binomial tree up to 2048 bytes, pre-fold + pairwise tree above) is bit-exact with every golden
case, every dtype and P = 2..8; the rank-order fold is bit-exact for integers, fp32 at P=2 and
exactly summable fp32, and within the summation bound |y - y_hat| <= (P-1) * u * sum_r |x_r|
(u = unit roundoff) otherwise.
"""
import json
import os

import numpy as np
import pytest

from _helpers import FROM_NP

HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = np.load(os.path.join(HERE, 'golden', 'golden_mpich.npz'), allow_pickle=False)
MANIFEST = json.load(open(os.path.join(HERE, 'golden', 'golden_manifest.json')))
CASES = sorted(MANIFEST['cases'])


def _bound(xs, dtype):
    """Largest difference between two summation orders of the same P terms: each is within
    (P-1) u sum|x| of the exact sum, so two of them are within twice that of each other."""
    u = np.finfo(dtype).eps / 2
    P = xs.shape[0]
    return 2 * (P - 1) * u * np.abs(xs.astype(np.float64)).sum(axis=0) * 1.0001


@pytest.mark.parametrize('case', CASES)
def test_oracle_matches_mpich(oracle, case):
    meta = MANIFEST['cases'][case]
    xs, y = GOLD[case + '__inputs'], GOLD[case + '__output']
    dt = FROM_NP[meta['dtype']]
    seq = oracle.allreduce_seq(dt, list(xs))
    exact = (np.issubdtype(xs.dtype, np.integer) or meta['P'] == 2 or meta['kind'] in
             ('exact', 'fill_rank', 'survey_probe'))
    if exact:
        assert seq.tobytes() == y.tobytes(), f'{case}: oracle != MPICH'
    else:
        err = np.abs(seq.astype(np.float64) - y.astype(np.float64))
        assert np.all(err <= _bound(xs, xs.dtype)), f'{case}: outside the summation bound'


@pytest.mark.parametrize('case', CASES)
def test_reference_order_is_bit_exact_with_mpich(oracle, case):
    """MPICH's summation order, restated (ddlo_fold_ref_order), reproduces MPI_Allreduce's output
    bit for bit — random fp32/fp64 at non-power-of-two P on both sides of the 2048-byte
    algorithm switch included."""
    meta = MANIFEST['cases'][case]
    xs, y = GOLD[case + '__inputs'], GOLD[case + '__output']
    got = oracle.fold_ref_order(FROM_NP[meta['dtype']], list(xs))
    assert got.tobytes() == y.tobytes(), f'{case}: {int((got != y).sum())} elements differ'


def test_reference_order_switch_is_what_distinguishes_p5(oracle):
    """At P=5 the two MPICH trees differ: each golden case matches exactly one of them, the one
    its message size selects (<= 2048 bytes: binomial)."""
    for case, small in (('fp32_randn_P5_small', True), ('fp32_randn_P5_switch', False)):
        xs, y = GOLD[case + '__inputs'], GOLD[case + '__output']
        tiny = oracle.fold_ref_order(1, list(xs), total_bytes=2048)
        big = oracle.fold_ref_order(1, list(xs), total_bytes=2049)
        assert (tiny.tobytes() == y.tobytes()) == small and (big.tobytes() == y.tobytes()) == (not small)


@pytest.mark.parametrize('P', [2, 4, 8])
def test_reference_test_known_answer(oracle, P):
    """src/py/ddl/test/allreduce_test.py:13 — fp32[16] filled with rank sums to P(P-1)/2."""
    xs = GOLD[f'ref_test_P{P}__inputs']
    y = oracle.allreduce_seq(1, list(xs))
    assert np.all(y == P * (P - 1) / 2)
    assert np.all(GOLD[f'ref_test_P{P}__output'] == P * (P - 1) / 2)


def test_survey_recorded_reference_outputs(oracle):
    """Spot values SURVEY.md §4 recorded from the reference's own C++ path."""
    rec = MANIFEST['survey_recorded']
    for P, tag in ((2, 'survey_probe_f32_P2'), (8, 'survey_probe_f32_P8')):
        y = oracle.allreduce_seq(1, list(GOLD[tag + '__inputs']))
        for i, v in rec[f'P{P}']['f32'].items():
            i = int(i)
            if i < y.size:
                assert y[i] == v
            else:  # beyond the stored 1024 elements: same generator, checked analytically
                assert sum(np.float32(0.5 * (r + 1) + (i % 7)) for r in range(P)) == v
    yi = oracle.allreduce_seq(3, list(GOLD['survey_probe_i32_P8__inputs']))
    assert yi[0] == rec['P8']['i32']['0']


def test_ring_order_equals_mpich_where_order_free(oracle, lib):
    """The ring-order restatement agrees with MPICH wherever the result is order-free."""
    from _helpers import ring_perms, ring_shape
    for case in ('int32_rand_P8', 'fp32_exact_P8', 'int32_rand_P4', 'fp32_randn_P2', 'uint64_rand_P2'):
        xs, y = GOLD[case + '__inputs'], GOLD[case + '__output']
        dt = FROM_NP[str(xs.dtype)]
        P = xs.shape[0]
        R, _ = ring_shape(lib, xs.shape[1], dt, P)
        out = oracle.allreduce_ring(dt, list(xs), ring_perms(lib, P, R))
        assert out.tobytes() == y.tobytes(), case


def test_half_and_bf16_rounding(oracle):
    """fp16/bf16 conversions of the oracle are round-to-nearest-even (numpy as the check)."""
    rng = np.random.default_rng(7)
    f = np.concatenate([rng.standard_normal(20000).astype(np.float32) * s for s in (1e-6, 1e-3, 1, 300, 6e4)])
    f = np.concatenate([f, np.array([65504, 65519.99, 65520, 6.1e-5, 5.96e-8, 2.98e-8, 0.0, -0.0], np.float32)])
    want = f.astype(np.float16).view(np.uint16)
    got = np.array([oracle.lib.ddlo_float_to_half(float(v)) for v in f], dtype=np.uint16)
    assert np.array_equal(got, want)
    h = np.arange(0, 65536, dtype=np.uint32).astype(np.uint16)
    h = h[(h & 0x7C00) != 0x7C00]  # finite halves
    back = np.array([oracle.lib.ddlo_half_to_float(int(v)) for v in h], dtype=np.float32)
    assert np.array_equal(back, h.view(np.float16).astype(np.float32))
    # bf16 sum = round_bf16(float(a) + float(b))
    u = f.view(np.uint32)
    rne = ((u.astype(np.uint64) + 0x7FFF + ((u >> 16) & 1)) >> 16).astype(np.uint16)
    got_bf = np.array([oracle.lib.ddlo_float_to_bf16(float(v)) for v in f[:5000]], dtype=np.uint16)
    assert np.array_equal(got_bf, rne[:5000])


@pytest.mark.parametrize('case', CASES)
def test_direct_order_vs_mpich(oracle, case):
    """The direct-schedule restatement (ddlo_allreduce_direct) against MPICH: bit-exact where
    the sum is order-free, within the summation bound otherwise (for fp16/bf16, which MPICH
    cannot reduce, the fold rounds once, so its error is the fp32 accumulation's)."""
    meta = MANIFEST['cases'][case]
    xs, y = GOLD[case + '__inputs'], GOLD[case + '__output']
    dt = FROM_NP[meta['dtype']]
    out = oracle.allreduce_direct(dt, list(xs))
    exact = (np.issubdtype(xs.dtype, np.integer) or meta['P'] == 2 or meta['kind'] in
             ('exact', 'fill_rank', 'survey_probe'))
    if exact:
        assert out.tobytes() == y.tobytes(), case
    else:
        err = np.abs(out.astype(np.float64) - y.astype(np.float64))
        assert np.all(err <= _bound(xs, xs.dtype)), case


def test_reference_broadcast_and_allgather_known_answers(oracle):
    """broadcast_test.py:5-17 (fp32[16] = rank + 1, root 3 -> 4 everywhere) and
    allgather_test.py:5-26 (IndexedSlices rows arange(4 + rank) + rank and
    [[0,0],..,[3,3]] + rank, gathered in rank order) through the oracle's restatements."""
    for P in (4, 8):
        xs = [np.full(16, r + 1, np.float32) for r in range(P)]
        for out in oracle.broadcast(1, xs, 3):
            assert np.all(out == 4)
    P = 3
    values = [np.arange(4 + r, dtype=np.float32) + r for r in range(P)]
    indices = [(np.array([[0, 0], [1, 1], [2, 2], [3, 3]]) + r).astype(np.float32) for r in range(P)]
    v, i = oracle.allgather_requests(1, [[a, b] for a, b in zip(values, indices)])
    assert v.tolist() == [0, 1, 2, 3, 1, 2, 3, 4, 5, 2, 3, 4, 5, 6, 7]
    assert i.tolist() == [[r + k, r + k] for r in range(P) for k in range(4)]
    assert np.array_equal(oracle.allgatherv(1, values), v)


def test_bench_parity_check_matches_mpich_golden(oracle):
    """bench.py's N>1 parity leg restates MPICH's order in numpy (mpich_order_sum); it must agree
    with MPICH's golden outputs and the oracle on every golden case (P = 2..8, both sides of the
    2048-byte switch)."""
    import importlib.util
    spec = importlib.util.spec_from_file_location('bench_mod', os.path.join(os.path.dirname(HERE), 'bench.py'))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    for case, meta in MANIFEST['cases'].items():
        xs, y = GOLD[case + '__inputs'], GOLD[case + '__output']
        got = bench.mpich_order_sum(list(xs), xs[0].nbytes)
        assert got.tobytes() == y.tobytes(), case


# ---- beyond one node's GPUs: P = 17 .. 520 on one host (tests/golden/make_golden.py --bigp) ----
GOLD_BIGP = np.load(os.path.join(HERE, 'golden', 'golden_mpich_bigp.npz'), allow_pickle=False)
MANIFEST_BIGP = json.load(open(os.path.join(HERE, 'golden', 'golden_manifest_bigp.json')))


@pytest.mark.parametrize('case', sorted(MANIFEST_BIGP['cases']))
def test_reference_order_bit_exact_with_mpich_beyond_8_ranks(oracle, case):
    """MPICH's order at P = 17, 20, 33 (non-power-of-two, both sides of 2048 bytes) and P = 520
    (count < pof2: recursive doubling above 2048 bytes) equals the oracle bit for bit."""
    meta = MANIFEST_BIGP['cases'][case]
    xs, y = GOLD_BIGP[case + '__inputs'], GOLD_BIGP[case + '__output']
    got = oracle.fold_ref_order(FROM_NP[meta['dtype']], list(xs))
    assert got.tobytes() == y.tobytes(), case


def test_count_below_pof2_rule_is_what_distinguishes_p520(oracle):
    """At P = 520 a 257-element fp64 message (2056 B) is above MPICH's 2048-byte switch, but its
    element count is below pof2 = 512, so MPICH reduces by recursive doubling: the size-only
    rule (pre-fold + pairwise tree) would differ from MPICH's output."""
    xs = list(GOLD_BIGP['fp64_randn_P520_count_lt_pof2__inputs'])
    y = GOLD_BIGP['fp64_randn_P520_count_lt_pof2__output']
    assert oracle.fold_ref_order(2, xs).tobytes() == y.tobytes()
    pof2 = 512
    rem = len(xs) - pof2
    leaf = [xs[2 * t] + xs[2 * t + 1] for t in range(rem)] + xs[2 * rem:]
    m = 1
    while m < pof2:
        for t in range(0, pof2, 2 * m):
            leaf[t] = leaf[t] + leaf[t + m]
        m *= 2
    assert leaf[0].tobytes() != y.tobytes()


@pytest.mark.parametrize('case', [c[0] for c in __import__('_helpers').fullsize_cases()])
def test_oracle_full_size_hash_matches_mpich(oracle, case):
    """C3 at its full size (P = 8, 64 Mi fp32 per rank) and the non-power-of-two pre-fold at that
    size (P = 5, 7): the oracle's MPICH order hashes to MPICH 3.3.2's own output (VERDICT r5 next
    #1; tests/golden/golden_fullsize.json, made by make_golden.py --fullsize)."""
    from _helpers import DT_FLOAT, fullsize_cases, fullsize_inputs, sha256
    name, P, n, digest, samples = next(c for c in fullsize_cases() if c[0] == case)
    xs = fullsize_inputs(P, n)
    y = oracle.fold_ref_order(DT_FLOAT, xs)
    del xs
    for i, v in samples.items():
        assert float(y[i]) == v, (case, i)
    assert sha256(y) == digest, case
