"""The ring schedule (host side of the engine, no GPU): ring construction, bucket partition,
per-rank programs and fusion plans — each checked against the oracle's restatement."""
import itertools

import numpy as np
import pytest

from _helpers import (ALL_DTYPES, DT_BFLOAT16, DT_FLOAT, DT_HALF, DT_INT32, GENERAL_FOLDS, config, NP, random_input,
                      ring_perms, ring_program, ring_shape, simulate_ring)

SZ_OF = {1: 4, 2: 8, 3: 4, 9: 8, 14: 2, 19: 2, 23: 8}


@pytest.fixture(autouse=True)
def _schedules_as_configured(lib):
    """Most tests here check the ring and the left-fold direct / one-shot schedules as built
    (reference_order 0); the reference-order tests opt back in."""
    with config(lib, reference_order=0):
        yield


@pytest.mark.parametrize('P', range(1, 9))
def test_rings_are_edge_disjoint_hamiltonian_cycles(lib, P):
    R = lib.ddl_ring_count(P, 8)
    expected = {1: 1, 2: 1, 3: 2, 4: 2, 5: 4, 6: 4, 7: 6, 8: 7}[P]
    assert R == expected  # P-1 except K4*/K6* (Tillson), natural ring only at P<=2
    perms = ring_perms(lib, P, R)
    assert perms[0] == list(range(P))  # ring 0 = the reference's token direction r -> r+1
    edges = set()
    for p in perms:
        assert sorted(p) == list(range(P))
        for i in range(P if P > 1 else 0):
            e = (p[i], p[(i + 1) % P])
            if P > 2:
                assert e not in edges
            edges.add(e)


@pytest.mark.parametrize('P', [9, 12, 16, 64])
def test_rings_beyond_one_node_are_stride_cycles(lib, P):
    """P > 8: rings r -> r + s for every s coprime to P (edge-disjoint Hamiltonian cycles),
    built constructively — the exhaustive search would enumerate (P-1)! cycles."""
    import math
    R = lib.ddl_ring_count(P, 8)
    assert R == min(8, sum(1 for s in range(1, P) if math.gcd(s, P) == 1))
    edges = set()
    for p in ring_perms(lib, P, R):
        assert sorted(p) == list(range(P))
        for i in range(P):
            e = (p[i], p[(i + 1) % P])
            assert e not in edges
            edges.add(e)


@pytest.mark.parametrize('n', [0, 1, 63, 64, 65, 1000, 4099, 1 << 16, 3 * (1 << 20) + 7])
@pytest.mark.parametrize('P', [2, 3, 4, 8])
@pytest.mark.parametrize('dt', [DT_FLOAT, DT_HALF, 2])
def test_chunk_partition_matches_oracle_and_tiles_bucket(lib, oracle, n, P, dt):
    import ctypes
    R, _ = ring_shape(lib, n, dt, P)
    es = SZ_OF[dt]
    covered = []
    for j in range(R):
        for c in range(P):
            b, e = ctypes.c_size_t(), ctypes.c_size_t()
            assert lib.ddl_chunk_range(n, dt, P, R, j, c, ctypes.byref(b), ctypes.byref(e)) == 0
            assert (b.value, e.value) == oracle.chunk_range(n, es, P, R, j, c)
            assert (b.value * es) % 256 == 0  # granule-aligned starts
            covered.append((b.value, e.value))
    pos = 0
    for b, e in covered:  # contiguous, in order, covering [0, n)
        assert b == pos or e <= b
        pos = max(pos, e)
    assert pos == n


@pytest.mark.parametrize('P', [2, 3, 4, 5, 8])
@pytest.mark.parametrize('n', [1, 100, 4099, 50_000])
@pytest.mark.parametrize('dt', ALL_DTYPES)
def test_ring_programs_compute_the_ring_order_sum(lib, oracle, P, n, dt):
    """All P per-rank programs, executed with matched sends/recvs, give the oracle's
    ring-order result bit for bit on every rank."""
    xs = [random_input(dt, n, 1234 + 7919 * r) for r in range(P)]
    outs = simulate_ring(oracle, lib, dt, xs)
    R, _ = ring_shape(lib, n, dt, P)
    want = oracle.allreduce_ring(dt, xs, ring_perms(lib, P, R))
    for r in range(P):
        assert outs[r].tobytes() == want.tobytes(), f'rank {r}'


def test_ring_program_slices_and_dependencies(lib):
    """Reduce-scatter ticks: every send of step s>0 waits on the reduce of step s-1 that produced
    it; staging offsets stay inside the staging buffer; each rank sends and receives the same
    byte volume 2(P-1)/P * S (the ring's wire cost)."""
    P, n, dt = 8, 256 << 20 >> 2, DT_FLOAT  # 256 MiB fp32 (C3)
    R, K = ring_shape(lib, n, dt, P)
    assert R == 7 and K >= 2
    for rank in range(P):
        prog = ring_program(lib, rank, P, n, dt)
        sent = prog[prog[:, 1] == 0][:, 6].sum()
        recv = prog[prog[:, 1] == 1][:, 6].sum()
        expect = 2 * (P - 1) * n / P
        assert abs(sent - expect) <= 2 * R * P * 64 and abs(recv - expect) <= 2 * R * P * 64
        rs_ticks = (P - 1) * K
        for row in prog[(prog[:, 1] == 0) & (prog[:, 0] < rs_ticks)]:
            t = row[0]
            if t >= K:
                assert row[7] == t - K and row[4] == 1  # forwards the previous step's output
            else:
                assert row[7] == -1 and row[4] == 0  # step 0 sends the rank's own input


def _overlap(a0, a1, b0, b1):
    return a0 < b1 and b0 < a1


@pytest.mark.parametrize('algo,ref_order', [(0, 0), (1, 0), (2, 0), (1, 1), (2, 1), (4, 0), (4, 1)])
@pytest.mark.parametrize('P', [2, 3, 4, 5, 7, 8, 17, 33])
@pytest.mark.parametrize('n', [777, 40_961, 1_000_003, (256 << 20) // 4 + 4096 * 3 + 5, 64 * 33 * 8 * 64])
@pytest.mark.parametrize('slice_bytes', [64 << 10, 2 << 20])
def test_schedule_has_no_stream_races(lib, algo, ref_order, P, n, slice_bytes):
    """Comm tick T runs after the reduce it waits on (W) and every earlier reduce (the compute
    stream is in order), but concurrently with the reduces of ticks W+1..T-1. None of T's
    sends/recvs may touch a buffer range those reduces read or write — with in and out treated
    as one buffer, since in-place allreduce (in == out) is allowed."""
    with config(lib, slice_bytes=slice_bytes, algo=algo, reference_order=ref_order):
        for rank in range(P):
            prog = ring_program(lib, rank, P, n, DT_FLOAT)
            red = {}
            for row in prog[(prog[:, 1] == 2) | (prog[:, 1] == 3)]:
                red.setdefault(int(row[0]), []).append(row)
            for row in prog[np.isin(prog[:, 1], list(GENERAL_FOLDS))]:  # general fold: reads (buf, off), writes out
                t_, kind_, _, _, sb, so, c_, oo = row
                ob = GENERAL_FOLDS[int(kind_)][1]  # 1: the output buffer, 2: a staging partial
                red.setdefault(int(t_), []).append(('gen', int(sb), int(so), int(c_), int(oo), ob))
            # an allgather (kind 11, direct-gather) as the send of its block and the receive of
            # all P blocks, with the tick's reduce wait
            gathers = []
            for g in prog[prog[:, 1] == 11]:
                t_, _, sb, so, rb, ro, c_, w_ = g
                gathers += [[t_, 0, -1, -1, sb, so, c_, w_], [t_, 1, -1, -1, rb, ro, P * c_, w_]]
            if gathers:
                prog = np.concatenate([prog, np.array(gathers, dtype=prog.dtype)])
            w_eff = -1  # the comm stream is in order: a tick inherits every earlier tick's wait
            for t in sorted(set(prog[:, 0].tolist())):
                ops = prog[(prog[:, 0] == t) & (prog[:, 1] <= 1)]
                if not len(ops):
                    continue
                w = int(ops[0][7])
                w = max([x for x in red if x <= w], default=-1) if w >= 0 else -1
                w_eff = max(w_eff, w)
                running = [r for tt, rows in red.items() if w_eff < tt < t for r in rows]
                for op in ops:
                    _, kind, _, _, buf, off, cnt, _ = op
                    for r in running:
                        if isinstance(r, tuple):  # general fold step: (tag, buffer, offset, count, out offset, out buffer)
                            _, sb, so, c_, oo, ob = r
                            rng_ = (so, so + c_) if sb == 2 else None
                            if buf == 2 and rng_:
                                assert not _overlap(off, off + cnt, *rng_), (rank, t, 'staging')
                            if buf == 2 and ob == 2:
                                assert not _overlap(off, off + cnt, oo, oo + c_), (rank, t, 'staging partial')
                            if buf != 2:
                                if ob == 1:
                                    assert not _overlap(off, off + cnt, oo, oo + c_), (rank, t, 'in/out')
                                if sb != 2:
                                    assert not _overlap(off, off + cnt, so, so + c_), (rank, t, 'in/out')
                            continue
                        _, _, _, _, _, roff, rcnt, soff = r
                        # a reduce reads in[roff:+rcnt] and staging[soff:+rcnt], writes out[roff:+rcnt]
                        if buf == 2:
                            assert not _overlap(off, off + cnt, soff, soff + rcnt), (rank, t, 'staging')
                        else:
                            assert not _overlap(off, off + cnt, roff, roff + rcnt), (rank, t, 'in/out')
                        if buf == 0 and kind == 1:
                            raise AssertionError('recv into the input buffer')


@pytest.mark.parametrize('P', [2, 3, 4, 5, 8])
@pytest.mark.parametrize('n', [1, 100, 4099, 50_000])
@pytest.mark.parametrize('dt', ALL_DTYPES)
def test_direct_programs_compute_the_direct_fold(lib, oracle, P, n, dt):
    """The direct (all-to-all) schedule: every rank's program, executed with matched
    sends/recvs, gives the oracle's direct fold bit for bit; for fp32/fp64/integers that is also
    the ring-0 order (fp16/bf16 accumulate in fp32 and round once)."""
    xs = [random_input(dt, n, 99 + 31 * r) for r in range(P)]
    with config(lib, algo=1):
        outs = simulate_ring(oracle, lib, dt, xs)
    want = oracle.allreduce_direct(dt, xs)
    for r in range(P):
        assert outs[r].tobytes() == want.tobytes(), f'rank {r}'
    if dt not in (DT_HALF, DT_BFLOAT16):
        assert want.tobytes() == oracle.allreduce_ring(dt, xs, [list(range(P))]).tobytes()


def test_direct_program_shape(lib):
    """Direct schedule at C3 (256 MiB fp32, P=8): K reduce-scatter ticks, each sending one slice
    to every peer and folding P-1 received inputs, then K allgather ticks; each rank moves
    2(P-1)/P * S bytes, like the ring, in 2K ticks instead of 2(P-1)K."""
    P, n = 8, 256 << 20 >> 2
    with config(lib, algo=1):
        R, K = ring_shape(lib, n, DT_FLOAT, P)
        assert R == 1 and K >= 2
        for rank in range(P):
            prog = ring_program(lib, rank, P, n, DT_FLOAT)
            assert int(prog[:, 0].max()) + 1 == 2 * K
            sent = prog[prog[:, 1] == 0][:, 6].sum()
            assert abs(sent - 2 * (P - 1) * n / P) <= 2 * P * P * 64
            folds = prog[prog[:, 1] == 3]
            assert len(folds) == K * (P - 1) and set(folds[:, 2]) == {P - 1}
            for row in prog[(prog[:, 1] == 0) & (prog[:, 0] >= K)]:
                assert row[7] == row[0] - K  # allgather slice k waits the fold of slice k


def test_plans_match_reference_plan_walk(lib, oracle):
    """makeCollectiveCommunicatePlan (MPIRingTokenCommunication.cc:495-546) restated in the
    oracle vs the engine's make_plans, on cases where the reference's walk is well defined
    (odd byte caps with even element sizes, as its 2^31-1 cap)."""
    import ctypes
    rng = np.random.default_rng(3)
    for trial in range(300):
        k = int(rng.integers(1, 12))
        esz = [int(rng.choice([2, 4, 8]))] * k  # one dtype group
        el = [int(rng.integers(0, 5000)) for _ in range(k)]
        el[0] = max(el[0], 1)
        limit = int(rng.integers(1, 40000)) | 1
        ref = oracle.make_plan(el, esz, limit)
        n = len(el)
        out = (ctypes.c_size_t * (4 * 8192))()
        np_ = ctypes.c_size_t()
        assert lib.ddl_make_plans((ctypes.c_size_t * n)(*el), (ctypes.c_size_t * n)(*esz), n, limit, out, 8192,
                                  ctypes.byref(np_)) == 0
        got = [tuple(out[4 * i:4 * i + 4]) for i in range(np_.value)]
        assert got == ref, (el, esz, limit)


def test_make_plans_even_cap_deliberate_divergence(lib, oracle):
    """An even cap can end a multi-request plan exactly on a request boundary. The reference then
    advances `requestPlannedBegin += 1` (MPIRingTokenCommunication.cc:534-536), so the next plan
    starts AGAIN at the request just finished — it is packed and reduced twice (in place, the
    second pass would add the already-reduced values). The engine continues after it
    (pe + 1). Hand-checked: 3 x fp32[4] (16 B each), cap 32 B."""
    import ctypes
    el, esz, cap = [4, 4, 4], [4, 4, 4], 32
    assert oracle.make_plan(el, esz, cap) == [(0, 0, 1, 4), (1, 0, 2, 4)]  # the reference's walk
    out = (ctypes.c_size_t * 64)()
    np_ = ctypes.c_size_t()
    assert lib.ddl_make_plans((ctypes.c_size_t * 3)(*el), (ctypes.c_size_t * 3)(*esz), 3, cap, out, 16,
                              ctypes.byref(np_)) == 0
    got = [tuple(out[4 * i:4 * i + 4]) for i in range(np_.value)]
    assert got == [(0, 0, 1, 4), (2, 0, 2, 4)]  # every request exactly once
    # with the reference's odd cap (2^31 - 1) and even element sizes the boundary case cannot
    # occur, and the two walks agree (test_make_plans_matches_oracle)


def test_plan_cap_2gib_single_plan_for_large_bucket(oracle):
    """With the reference's cap (2^31-1 bytes) a 256 MiB fp32 bucket is one plan (C3), and a
    C5-like mixed set splits where the reference would."""
    cap = (1 << 31) - 1
    assert oracle.make_plan([64 << 20], [4], cap) == [(0, 0, 0, 64 << 20)]
    el = [600 << 20 >> 2] * 4  # 4 x 600 MiB fp32 -> 2.34 GiB -> two plans
    plans = oracle.make_plan(el, [4] * 4, cap)
    assert len(plans) == 2 and plans[0][2] == 3 and plans[1][0] == 3


def test_token_key_order_is_bytewise_lexicographic():
    """std::set<pair<string,string>> order (RingTokenCommunicateHandler.cc:365-400) is bytewise:
    the engine keeps pending requests in a std::map<std::string,...> — same order as Python
    sorting of bytes keys."""
    keys = [b'grad_00010', b'grad_9', b'Grad_1', b'grad_\xc3\xa9', b'grad_0001']
    assert sorted(keys) == [b'Grad_1', b'grad_0001', b'grad_00010', b'grad_9', b'grad_\xc3\xa9']


def test_direct_program_sixteen_ranks(lib, oracle):
    """The direct fold's widest case (15 received inputs, the kernel's limit) builds at once and
    computes the direct-fold sum."""
    P, n = 16, 5000
    xs = [random_input(DT_HALF, n, 3 + r) for r in range(P)]
    with config(lib, algo=1):
        outs = simulate_ring(oracle, lib, DT_HALF, xs)
    want = oracle.allreduce_direct(DT_HALF, xs)
    assert all(o.tobytes() == want.tobytes() for o in outs)


@pytest.mark.parametrize('P', [2, 3, 4, 5, 8, 16])
@pytest.mark.parametrize('n', [1, 100, 4099, 50_000])
@pytest.mark.parametrize('dt', ALL_DTYPES)
def test_oneshot_programs_compute_the_rank_order_fold(lib, oracle, P, n, dt):
    """One-shot schedule (algo 2): one group exchanging whole buckets with every peer, then a
    fold of the P inputs in rank order 0..P-1 on every rank: every rank holds the oracle's
    rank-order fold bit for bit (identical on all ranks; fp16/bf16 accumulated in fp32)."""
    xs = [random_input(dt, n, 7 + 13 * r) for r in range(P)]
    with config(lib, algo=2):
        outs = simulate_ring(oracle, lib, dt, xs)
    want = oracle.fold(dt, xs)
    for r in range(P):
        assert outs[r].tobytes() == want.tobytes(), f'rank {r}'


def test_oneshot_program_shape(lib):
    """One tick of 2(P-1) whole-bucket p2p ops, one (P-1)-input fold, and a trailing tick that
    waits for the fold (so the caller's join covers it); staging of P-1 buckets."""
    P, n = 8, 1 << 16
    with config(lib, algo=2):
        for rank in range(P):
            prog = ring_program(lib, rank, P, n, DT_FLOAT)
            ops = prog[prog[:, 1] <= 1]
            assert set(ops[:, 0]) == {0} and len(ops) == 2 * (P - 1) and set(ops[:, 6]) == {n}
            assert sorted(ops[ops[:, 1] == 0][:, 2]) == sorted(set(range(P)) - {rank})
            folds = prog[(prog[:, 1] == 3) | np.isin(prog[:, 1], list(GENERAL_FOLDS))]
            assert set(folds[:, 0]) == {0}


# ---- reference order (reference_order = 1, the default) ----------------------------------------
@pytest.mark.parametrize('algo', [0, 1, 2, 3, 4])
@pytest.mark.parametrize('P', [2, 3, 4, 5, 6, 7, 8])
@pytest.mark.parametrize('n', [1, 100, 512, 513, 4099, 50_000, 128 * 840])
@pytest.mark.parametrize('dt', ALL_DTYPES)
def test_reference_order_programs_compute_mpich_order(lib, oracle, algo, P, n, dt):
    """With reference_order every schedule's programs, executed with matched sends/recvs, give
    MPICH 3.3.2's own MPI_Allreduce order on every rank, bit for bit: the oracle's
    ddlo_fold_ref_order (pinned to MPICH runs by test_oracle_golden), binomial tree for
    messages <= 2048 bytes and pre-fold + pairwise tree above. A ring at P > 2 runs as the direct
    schedule; a P = 2 ring is order-free. fp16 / bf16 (rejected by the reference) fold in rank
    order in fp32."""
    xs = [random_input(dt, n, 11 + 29 * r) for r in range(P)]
    with config(lib, algo=algo, reference_order=1):
        outs = simulate_ring(oracle, lib, dt, xs)
    want = oracle.fold_ref_order(dt, xs)
    for r in range(P):
        assert outs[r].tobytes() == want.tobytes(), f'rank {r}'


@pytest.mark.parametrize('P', [2, 3, 5, 8])
def test_direct_gather_program_shape(lib, P):
    """Direct-gather (algo 4): the direct reduce-scatter ticks, then ONE in-place allgather of the
    reduced chunks (kind 11, send = out at rank * n / P, recv = out, n / P per rank) waiting for
    the last fold — where the chunks are equal; elsewhere the direct program itself."""
    n = 128 * 840  # fp32: 430080 B = 1680 granules, a multiple of every P here
    with config(lib, algo=1, reference_order=1, slice_bytes=64 << 10):
        direct = [ring_program(lib, r, P, n, DT_FLOAT) for r in range(P)]
        ragged = [ring_program(lib, r, P, n + 64, DT_FLOAT) for r in range(P)]
    with config(lib, algo=4, reference_order=1, slice_bytes=64 << 10):
        progs = [ring_program(lib, r, P, n, DT_FLOAT) for r in range(P)]
        ragged4 = [ring_program(lib, r, P, n + 64, DT_FLOAT) for r in range(P)]
    for r in range(P):
        g = progs[r][progs[r][:, 1] == 11]
        assert len(g) == 1
        t, _, sb, so, rb, ro, cnt, wait = g[0]
        assert (sb, so, rb, ro, cnt) == (1, r * n // P, 1, 0, n // P)
        assert t == progs[r][:, 0].max() and not ((progs[r][:, 0] == t) & (progs[r][:, 1] <= 1)).any()
        rs = direct[r][direct[r][:, 0] < t]
        assert np.array_equal(progs[r][progs[r][:, 0] < t], rs)  # the same reduce-scatter
        assert wait == rs[rs[:, 1] <= 1][:, 0].max()  # the last reduce-scatter tick's fold
        assert np.array_equal(ragged4[r], ragged[r])  # unequal chunks: the direct program


def test_reference_order_program_kinds(lib):
    """The fold rows name MPICH's algorithm by the message size: kind 7 (binomial) up to 2048
    bytes, kind 6 (pre-fold + pairwise tree) above; a ring asked for at P > 2 is the direct
    schedule (R = 1, 2K ticks); at P = 2 it stays the ring."""
    with config(lib, algo=0, reference_order=1):
        assert ring_shape(lib, 1 << 20, DT_FLOAT, 8)[0] == 1
        assert ring_shape(lib, 1 << 20, DT_FLOAT, 2)[0] == 1
        for n, kind in ((512, 7), (513, 6), (1 << 20, 6)):
            prog = ring_program(lib, 3, 5, n, DT_FLOAT)
            assert set(prog[prog[:, 1] >= 3][:, 1]) == {kind}, n
            assert set(prog[prog[:, 1] >= 3][:, 2]) == {5}  # every input named, rank order
        prog = ring_program(lib, 0, 2, 1 << 20, DT_FLOAT)
        assert set(prog[:, 1]) <= {0, 1, 2}  # ring: two-input reduces only
    with config(lib, algo=2, reference_order=1):
        prog = ring_program(lib, 2, 5, 300, DT_FLOAT)
        assert set(prog[prog[:, 1] >= 3][:, 1]) == {7}


@pytest.mark.parametrize('algo,ref_order', [(0, 1), (1, 1), (2, 1), (3, 1), (1, 0), (2, 0), (3, 0)])
@pytest.mark.parametrize('P', [17, 20, 31, 32, 33])
@pytest.mark.parametrize('n', [1, 300, 513, 5000])
@pytest.mark.parametrize('dt', [1, 2, 3, 19])
def test_fold_trees_beyond_sixteen_ranks(lib, oracle, algo, ref_order, P, n, dt):
    """Beyond 16 ranks one fold launch cannot take every input: the fold runs as a chain (left)
    or a tree of 16-input steps through staging partials (MPICH's orders), and must still give
    the exact sum of the requested order — MPICH's with reference_order (a ring runs as direct),
    else the left fold. fp16 (not in the reference) rounds once per 16-input step."""
    xs = [random_input(dt, n, 3 + 17 * r) for r in range(P)]
    with config(lib, algo=algo, reference_order=ref_order):
        outs = simulate_ring(oracle, lib, dt, xs)
    if dt == 19:
        want = None
    elif ref_order:
        want = oracle.fold_ref_order(dt, xs)
    elif algo == 1:
        want = oracle.allreduce_direct(dt, xs)
    else:
        want = oracle.fold(dt, xs)
    if want is None:  # fp16: identical on every rank and within the fp16 summation bound
        exact = np.sum([x.astype(np.float64) for x in xs], axis=0)
        bound = P * 2.0 ** -11 * np.sum([np.abs(x.astype(np.float64)) for x in xs], axis=0) + 2.0 ** -14
        for r in range(P):
            assert outs[r].tobytes() == outs[0].tobytes()
        assert np.all(np.abs(outs[0].astype(np.float64) - exact) <= bound)
        return
    for r in range(P):
        assert outs[r].tobytes() == want.tobytes(), f'rank {r}'


def test_fold_tree_shape_beyond_sixteen_ranks(lib):
    """P = 33, reference order, > 2048 bytes: one pre-fold step (rem = 1), then binomial blocks
    of 16 leaves into staging partials, then the top; every step has at most 16 inputs."""
    with config(lib, algo=1, reference_order=1):
        prog = ring_program(lib, 5, 33, 100_000, DT_FLOAT)
    gen = prog[np.isin(prog[:, 1], list(GENERAL_FOLDS))]
    assert gen[:, 2].max() <= 16
    t0 = gen[gen[:, 0] == gen[0, 0]]
    sizes, kinds, i = [], [], 0
    while i < len(t0):
        sizes.append(int(t0[i, 2]))
        kinds.append(int(t0[i, 1]))
        i += sizes[-1]
    assert sizes == [2, 16, 16, 2] and kinds == [8, 10, 10, 7], (sizes, kinds)


def test_random_schedules_property(lib, oracle):
    """Property check over random (P, n, dtype, algo, reference_order, slice_bytes, max_slices,
    rings): every rank's program, executed with matched sends/recvs, ends with the sum the
    configuration promises — MPICH's order with reference_order, else the ring / left-fold /
    rank-order fold — bit for bit."""
    rng = np.random.default_rng(2024)
    for trial in range(120):
        P = int(rng.integers(2, 9))
        n = int(rng.choice([1, 2, 63, 64, 65, 257, 511, 512, 513, 1000, 4099, 33_333, 100_003]))
        dt = int(rng.choice(ALL_DTYPES))
        algo = int(rng.integers(0, 3))
        ref = int(rng.integers(0, 2))
        kv = dict(algo=algo, reference_order=ref, slice_bytes=int(rng.choice([1 << 10, 64 << 10, 2 << 20])),
                  max_slices=int(rng.integers(1, 17)), rings=int(rng.integers(1, 9)))
        xs = [random_input(dt, n, 3 * trial + r) for r in range(P)]
        with config(lib, **kv):
            outs = simulate_ring(oracle, lib, dt, xs)
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


def _bigp_golden():
    import json
    import os
    here = os.path.dirname(os.path.abspath(__file__))
    gold = np.load(os.path.join(here, 'golden', 'golden_mpich_bigp.npz'), allow_pickle=False)
    meta = json.load(open(os.path.join(here, 'golden', 'golden_manifest_bigp.json')))['cases']
    return [(c, m, gold[c + '__inputs'], gold[c + '__output']) for c, m in sorted(meta.items())]


@pytest.mark.parametrize('case,meta,xs,y', _bigp_golden(), ids=[c for c, *_ in _bigp_golden()])
def test_programs_equal_mpich_beyond_8_ranks(lib, oracle, case, meta, xs, y):
    """The engine's own programs at P = 17 .. 520 (one host's MPICH outputs, tests/golden):
    executed with matched sends/recvs, every rank equals MPI_Allreduce bit for bit — the direct
    schedule at every P (fold trees of up to 520 inputs in <= 16-input steps; MPICH's
    count < pof2 rule at P = 520), one-shot and gather-fold up to 33 ranks."""
    from _helpers import FROM_NP
    dt = FROM_NP[meta['dtype']]
    for algo in ((1, 2, 3) if meta['P'] <= 33 else (1,)):
        with config(lib, algo=algo, reference_order=1):
            outs = simulate_ring(oracle, lib, dt, list(xs))
        for r, o in enumerate(outs):
            assert o.tobytes() == y.tobytes(), (algo, r)
