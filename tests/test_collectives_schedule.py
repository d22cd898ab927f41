"""Broadcast and allgather schedules (host side, no GPU): every rank's program from the engine
(ddl_broadcast_program / ddl_allgather_program), executed with matched sends/recvs, must
produce the oracle's MPI_Bcast / MPI_Allgatherv result (MPICommunicator.cc:31-90) bit for bit,
and the broadcast must move 2S/P per root link rather than S."""
import ctypes

import numpy as np
import pytest

from _helpers import (ALL_DTYPES, DT_FLOAT, DT_HALF, NP, SZ, config, program, random_input, simulate_moves)


@pytest.mark.parametrize('P', [1, 2, 3, 4, 5, 8])
@pytest.mark.parametrize('n', [0, 1, 100, 4099, 300_001])
@pytest.mark.parametrize('dt', [DT_FLOAT, DT_HALF, 9])
def test_broadcast_programs(lib, oracle, P, n, dt):
    for root in sorted({0, P - 1, P // 2}):
        xs = [random_input(dt, n, 50 + r) for r in range(P)]
        with config(lib, slice_bytes=64 << 10):
            progs = [program(lib, 'ddl_broadcast_program', r, P, root, n, dt) for r in range(P)]
        bufs = simulate_moves(progs, [[np.zeros(0, dtype=x.dtype), x.copy()] for x in xs])
        want = oracle.broadcast(dt, xs, root)
        for r in range(P):
            assert bufs[r][1].tobytes() == want[r].tobytes(), (root, r)
        if P > 1 and n:
            # per link: the root sends chunk c to rank c (scatter) and its own chunk once per peer
            root_sent = progs[root][progs[root][:, 1] == 0]
            per_peer = {int(q): int(root_sent[root_sent[:, 2] == q][:, 6].sum()) for q in range(P) if q != root}
            G = 256 // np.dtype(NP[dt]).itemsize
            assert max(per_peer.values()) <= 2 * (-(-n // P) + G)


def test_broadcast_pipelines_scatter_and_allgather(lib):
    """Tick t carries the scatter of slice t and the allgather of slice t-1 (K+1 ticks)."""
    P, n = 8, 64 << 20
    with config(lib, slice_bytes=2 << 20, max_slices=8):
        prog = program(lib, 'ddl_broadcast_program', 3, P, 0, n, DT_FLOAT)
    ticks = sorted(set(prog[:, 0].tolist()))
    assert len(ticks) == 9
    for t in ticks[1:-1]:
        tags = set(prog[prog[:, 0] == t][:, 3].tolist())
        assert tags == {0, 1}


@pytest.mark.parametrize('P', [1, 2, 3, 5, 8])
@pytest.mark.parametrize('dt', ALL_DTYPES)
def test_allgatherv_programs(lib, oracle, P, dt):
    rng = np.random.default_rng(P * 100 + dt)
    counts = [int(c) for c in rng.integers(0, 3000, size=P)]
    if P > 1:
        counts[1] = 0  # an empty contribution
    displs = list(np.cumsum([0] + counts[:-1]))
    total = sum(counts)
    sends = [random_input(dt, c, 7 + q) for q, c in enumerate(counts)]
    C = (SZ * P)(*counts)
    D = (SZ * P)(*[int(d) for d in displs])
    progs = [program(lib, 'ddl_allgather_program', r, P, C, D, dt) for r in range(P)]
    bufs = simulate_moves(progs, [[s.copy(), np.zeros(total, dtype=s.dtype)] for s in sends])
    want = oracle.allgatherv(dt, sends)
    for r in range(P):
        assert bufs[r][1].tobytes() == want.tobytes(), r


def test_allgatherv_strided_displacements_and_in_place(lib, oracle):
    """Non-packed displacements (gaps) and an in-place contribution (send already at its
    displacement inside recv: no copy row)."""
    P, dt = 4, DT_FLOAT
    counts = [5, 300, 0, 64]
    displs = [1000, 0, 500, 600]
    C, D = (SZ * P)(*counts), (SZ * P)(*displs)
    sends = [random_input(dt, c, q) for q, c in enumerate(counts)]
    progs = [program(lib, 'ddl_allgather_program', r, P, C, D, dt) for r in range(P)]
    for r in range(P):
        copies = progs[r][progs[r][:, 1] == 4]
        assert len(copies) == (1 if counts[r] else 0)
    bufs = simulate_moves(progs, [[s.copy(), np.zeros(1005, dtype=np.float32)] for s in sends])
    want = oracle.allgatherv(dt, sends, displs=displs, total=1005)
    assert all(b[1].tobytes() == want.tobytes() for b in bufs)


def test_allgather_requests_oracle_layout(oracle):
    """allgatherRequests output (MPIRingTokenCommunication.cc:338-356): per request, the ranks'
    rows concatenated in rank order (first dims may differ per rank)."""
    P = 3
    per_rank = [[np.full((q + 1, 2), 10 * q + j, np.float32) for j in range(2)] for q in range(P)]
    outs = oracle.allgather_requests(1, per_rank)
    assert outs[0].shape == (6, 2) and outs[1].shape == (6, 2)
    assert outs[1][:, 0].tolist() == [1, 11, 11, 21, 21, 21]
