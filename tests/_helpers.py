"""Test helpers: ctypes wrapper of the oracle (oracle/ddl_oracle.c) and data generators.

The oracle is the checker only; nothing here is imported by the product.
"""
import contextlib
import ctypes
import os

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_LIB = os.path.join(ROOT, 'oracle', 'build', 'libddl_oracle.so')

DT_FLOAT, DT_DOUBLE, DT_INT32, DT_INT64, DT_BFLOAT16, DT_HALF, DT_UINT64 = 1, 2, 3, 9, 14, 19, 23
# numpy storage type per dtype code (bf16 is stored as raw uint16)
NP = {DT_FLOAT: np.float32, DT_DOUBLE: np.float64, DT_INT32: np.int32, DT_INT64: np.int64,
      DT_HALF: np.float16, DT_BFLOAT16: np.uint16, DT_UINT64: np.uint64}
NAME = {DT_FLOAT: 'float32', DT_DOUBLE: 'float64', DT_INT32: 'int32', DT_INT64: 'int64',
        DT_HALF: 'float16', DT_BFLOAT16: 'bfloat16', DT_UINT64: 'uint64'}
ALL_DTYPES = [DT_FLOAT, DT_DOUBLE, DT_INT32, DT_INT64, DT_HALF, DT_BFLOAT16, DT_UINT64]
FROM_NP = {'float32': DT_FLOAT, 'float64': DT_DOUBLE, 'int32': DT_INT32, 'int64': DT_INT64,
           'uint64': DT_UINT64, 'float16': DT_HALF}

SZ = ctypes.c_size_t


def ptr(a: np.ndarray):
    return ctypes.c_void_p(a.ctypes.data)


class Oracle:
    def __init__(self, path=ORACLE_LIB):
        self.lib = L = ctypes.CDLL(path)
        L.ddlo_sum2.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, SZ]
        L.ddlo_allreduce_seq.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_void_p),
                                         ctypes.c_void_p, SZ]
        L.ddlo_allreduce_ring.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_int),
                                          ctypes.POINTER(ctypes.c_void_p), ctypes.c_void_p, SZ]
        L.ddlo_allreduce_direct.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_void_p),
                                            ctypes.c_void_p, SZ]
        L.ddlo_fold.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.POINTER(ctypes.c_void_p), ctypes.c_int, SZ]
        L.ddlo_fold_ref_order.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.POINTER(ctypes.c_void_p), ctypes.c_int,
                                          SZ, SZ]
        PV = ctypes.POINTER(ctypes.c_void_p)
        L.ddlo_broadcast.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, PV, SZ]
        L.ddlo_allgatherv.argtypes = [ctypes.c_int, ctypes.c_int, PV, ctypes.POINTER(SZ), ctypes.POINTER(SZ),
                                      ctypes.c_void_p]
        L.ddlo_allgather_requests.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.POINTER(SZ),
                                              ctypes.POINTER(SZ), PV, PV]
        L.ddlo_chunk_range.argtypes = [SZ, SZ, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                       ctypes.POINTER(SZ), ctypes.POINTER(SZ)]
        L.ddlo_make_plan.argtypes = [ctypes.POINTER(SZ), ctypes.POINTER(SZ), SZ, SZ, ctypes.POINTER(SZ), SZ]
        L.ddlo_make_plan.restype = ctypes.c_long
        L.ddlo_dtype_size.argtypes = [ctypes.c_int]
        L.ddlo_dtype_size.restype = SZ
        L.ddlo_reduce_reps.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, SZ, ctypes.c_int]
        L.ddlo_half_to_float.argtypes = [ctypes.c_uint16]
        L.ddlo_half_to_float.restype = ctypes.c_float
        L.ddlo_float_to_half.argtypes = [ctypes.c_float]
        L.ddlo_float_to_half.restype = ctypes.c_uint16
        L.ddlo_float_to_bf16.argtypes = [ctypes.c_float]
        L.ddlo_float_to_bf16.restype = ctypes.c_uint16

    def sum2(self, dt, a, b):
        a = np.ascontiguousarray(a)
        b = np.ascontiguousarray(b)
        out = np.empty_like(a)
        assert self.lib.ddlo_sum2(dt, ptr(out), ptr(a), ptr(b), a.size) == 0
        return out

    def allreduce_seq(self, dt, xs):
        xs = [np.ascontiguousarray(x) for x in xs]
        out = np.empty_like(xs[0])
        arr = (ctypes.c_void_p * len(xs))(*[x.ctypes.data for x in xs])
        assert self.lib.ddlo_allreduce_seq(dt, len(xs), arr, ptr(out), xs[0].size) == 0
        return out

    def allreduce_ring(self, dt, xs, perms):
        xs = [np.ascontiguousarray(x) for x in xs]
        P, R = len(xs), len(perms)
        flat = (ctypes.c_int * (P * R))(*[v for p in perms for v in p])
        out = np.empty_like(xs[0])
        arr = (ctypes.c_void_p * P)(*[x.ctypes.data for x in xs])
        assert self.lib.ddlo_allreduce_ring(dt, P, R, flat, arr, ptr(out), xs[0].size) == 0
        return out

    def allreduce_direct(self, dt, xs):
        xs = [np.ascontiguousarray(x) for x in xs]
        out = np.empty_like(xs[0])
        arr = (ctypes.c_void_p * len(xs))(*[x.ctypes.data for x in xs])
        assert self.lib.ddlo_allreduce_direct(dt, len(xs), arr, ptr(out), xs[0].size) == 0
        return out

    def fold(self, dt, xs):
        xs = [np.ascontiguousarray(x) for x in xs]
        out = np.empty_like(xs[0])
        arr = (ctypes.c_void_p * len(xs))(*[x.ctypes.data for x in xs])
        assert self.lib.ddlo_fold(dt, ptr(out), arr, len(xs), xs[0].size) == 0
        return out

    def fold_ref_order(self, dt, xs, total_bytes=None):
        """Sum of xs (rank order) in MPICH 3.3.2's MPI_Allreduce order for a message of
        total_bytes (default: the whole of one input)."""
        xs = [np.ascontiguousarray(x) for x in xs]
        out = np.empty_like(xs[0])
        arr = (ctypes.c_void_p * len(xs))(*[x.ctypes.data for x in xs])
        tb = xs[0].nbytes if total_bytes is None else total_bytes
        assert self.lib.ddlo_fold_ref_order(dt, ptr(out), arr, len(xs), xs[0].size, tb) == 0
        return out

    def broadcast(self, dt, xs, root):
        outs = [np.ascontiguousarray(x).copy() for x in xs]
        arr = (ctypes.c_void_p * len(outs))(*[o.ctypes.data for o in outs])
        assert self.lib.ddlo_broadcast(dt, len(outs), root, arr, outs[0].size) == 0
        return outs

    def allgatherv(self, dt, sends, displs=None, total=None):
        """Every rank's recv buffer (identical): send_q at displs[q] (default: packed)."""
        sends = [np.ascontiguousarray(x) for x in sends]
        counts = [x.size for x in sends]
        if displs is None:
            displs = list(np.cumsum([0] + counts[:-1]))
        if total is None:
            total = max([d + c for d, c in zip(displs, counts)], default=0)
        recv = np.zeros(total, dtype=sends[0].dtype)
        arr = (ctypes.c_void_p * len(sends))(*[x.ctypes.data for x in sends])
        assert self.lib.ddlo_allgatherv(dt, len(sends), arr, (SZ * len(sends))(*counts),
                                        (SZ * len(sends))(*[int(d) for d in displs]), ptr(recv)) == 0
        return recv

    def allgather_requests(self, dt, per_rank):
        """per_rank[q][j]: rank q's request j as a 2-D array (rows, row_elems)."""
        P, nreq = len(per_rank), len(per_rank[0])
        fd = [per_rank[q][j].shape[0] for q in range(P) for j in range(nreq)]
        re = [int(np.prod(per_rank[0][j].shape[1:])) for j in range(nreq)]
        ins = [np.ascontiguousarray(per_rank[q][j]) for q in range(P) for j in range(nreq)]
        outs = [np.zeros((sum(per_rank[q][j].shape[0] for q in range(P)),) + per_rank[0][j].shape[1:],
                         dtype=per_rank[0][j].dtype) for j in range(nreq)]
        ia = (ctypes.c_void_p * len(ins))(*[x.ctypes.data for x in ins])
        oa = (ctypes.c_void_p * max(1, nreq))(*[o.ctypes.data for o in outs])
        assert self.lib.ddlo_allgather_requests(dt, P, nreq, (SZ * len(fd))(*fd), (SZ * max(1, nreq))(*re), ia,
                                                oa) == 0
        return outs

    def chunk_range(self, n, esize, P, R, ring, chunk):
        b, e = SZ(), SZ()
        assert self.lib.ddlo_chunk_range(n, esize, P, R, ring, chunk, ctypes.byref(b), ctypes.byref(e)) == 0
        return b.value, e.value

    def make_plan(self, elements, esizes, limit, max_plans=4096):
        n = len(elements)
        el = (SZ * n)(*elements)
        es = (SZ * n)(*esizes)
        out = (SZ * (4 * max_plans))()
        k = self.lib.ddlo_make_plan(el, es, n, limit, out, max_plans)
        assert k >= 0
        return [tuple(out[4 * i:4 * i + 4]) for i in range(k)]


@contextlib.contextmanager
def config(lib, **kv):
    """Temporarily set engine tunables (ddl_set_config) and restore them."""
    old = {k: lib.ddl_get_config(k.encode()) for k in kv}
    try:
        for k, v in kv.items():
            assert lib.ddl_set_config(k.encode(), v) == 0
        yield
    finally:
        for k, v in old.items():
            lib.ddl_set_config(k.encode(), v)


def random_input(dt, n, seed, kind='randn'):
    """Seeded synthetic gradient bucket of dtype code dt."""
    rng = np.random.default_rng(seed)
    if dt in (DT_INT32, DT_INT64, DT_UINT64):
        info = np.iinfo(NP[dt])
        return rng.integers(info.min, info.max, size=n, dtype=NP[dt], endpoint=True)
    if kind == 'exact':  # k * 2^-10, |k| < 2^12: sums of up to 2^11 terms are exact in fp32
        k = rng.integers(-(2 ** 12) + 1, 2 ** 12, size=n)
        x = k * 2.0 ** -10
    else:
        x = rng.standard_normal(n)
    if dt == DT_BFLOAT16:
        f = x.astype(np.float32).view(np.uint32)
        return ((f + 0x7FFF + ((f >> 16) & 1)) >> 16).astype(np.uint16)
    if dt == DT_HALF:
        return (0.25 * x).astype(np.float16)
    return x.astype(NP[dt])


def ring_perms(lib, P, R, max_rings=8):
    perms = []
    buf = (ctypes.c_int * P)()
    for j in range(R):
        assert lib.ddl_ring_perm(P, max_rings, j, buf) == 0
        perms.append(list(buf))
    return perms


def ring_shape(lib, n, dt, P):
    r, k = ctypes.c_int(), ctypes.c_int()
    assert lib.ddl_ring_shape(n, dt, P, ctypes.byref(r), ctypes.byref(k)) == 0
    return r.value, k.value


def ring_program(lib, rank, P, n, dt):
    cap = 1 << 16
    buf = (ctypes.c_longlong * (8 * cap))()
    nops = SZ()
    st = lib.ddl_ring_program(rank, P, n, dt, buf, cap, ctypes.byref(nops))
    assert st == 0, lib.ddl_last_error()
    return np.frombuffer(buf, dtype=np.int64, count=8 * nops.value).reshape(-1, 8).copy()


def program(lib, fn, *args):
    """Rows of a program dump entry (ddl_ring_program / ddl_broadcast_program / ...)."""
    cap = 1 << 16
    buf = (ctypes.c_longlong * (8 * cap))()
    nops = SZ()
    st = getattr(lib, fn)(*args, buf, cap, ctypes.byref(nops))
    assert st == 0, lib.ddl_last_error()
    return np.frombuffer(buf, dtype=np.int64, count=8 * nops.value).reshape(-1, 8).copy()


def simulate_moves(progs, bufs):
    """Run data-movement-only programs (copies and matched sends/recvs, no reduces):
    bufs[r] = [buffer 0, buffer 1] of rank r; a send and a recv match on (tick, pair, tag) in
    posting order, as RCCL matches p2p operations of a group."""
    P = len(progs)
    T = int(max((p[:, 0].max() for p in progs if len(p)), default=-1)) + 1
    for t in range(T):
        for r in range(P):
            for row in progs[r][(progs[r][:, 0] == t) & (progs[r][:, 1] == 4)]:
                _, _, _, _, b, off, cnt, soff = row
                bufs[r][b][off:off + cnt] = bufs[r][0][soff:soff + cnt]
        sends = {}
        for r in range(P):
            for row in progs[r][(progs[r][:, 0] == t) & (progs[r][:, 1] == 0)]:
                _, _, peer, tag, b, off, cnt, _ = row
                sends.setdefault((r, peer, tag), []).append(bufs[r][b][off:off + cnt].copy())
        for r in range(P):
            for row in progs[r][(progs[r][:, 0] == t) & (progs[r][:, 1] == 1)]:
                _, _, peer, tag, b, off, cnt, _ = row
                data = sends[(peer, r, tag)].pop(0)
                assert data.size == cnt
                bufs[r][b][off:off + cnt] = data
        assert all(not v for v in sends.values()), f'unmatched sends at tick {t}'
    return bufs


def staging_size(progs, P=None):
    """Elements of staging a set of program dumps touches (recv targets, fold inputs/outputs);
    P = the number of ranks (default: one program per rank)."""
    P = len(progs) if P is None else P
    st_size = 1
    for p in progs:
        for row in p:
            if row[1] in (0, 1) and row[4] == 2:
                st_size = max(st_size, int(row[5] + row[6]))
            elif row[1] == 4 and row[4] == 2:  # copy into staging
                st_size = max(st_size, int(row[5] + row[6]))
            elif row[1] == 11:  # gather: P blocks of row[6] elements into (row[4], row[5])
                if row[4] == 2:
                    st_size = max(st_size, int(row[5] + P * row[6]))
                if row[2] == 2:  # sent from a (padded) staging slot
                    st_size = max(st_size, int(row[3] + row[6]))
            elif row[1] in (2, 3):
                st_size = max(st_size, int(row[7] + row[6]))
            elif row[1] in GENERAL_FOLDS:
                if row[4] == 2:
                    st_size = max(st_size, int(row[5] + row[6]))
                if GENERAL_FOLDS[int(row[1])][1] == 2:
                    st_size = max(st_size, int(row[7] + row[6]))
    return st_size


def simulate_ring(oracle, lib, dt, xs):
    """Execute every rank's ring (or direct) program, taken from the engine's own schedule, on
    host buffers: sends/recvs matched by (tick, peer, tag), 2-input reduces and N-input folds
    through the oracle's operators."""
    P, n = len(xs), xs[0].size
    progs = [ring_program(lib, r, P, n, dt) for r in range(P)]
    st_size = staging_size(progs)
    bufs = [[x.copy(), np.zeros_like(x), np.zeros(st_size, dtype=x.dtype)] for x in xs]
    T = int(max(p[:, 0].max() for p in progs)) + 1 if P > 1 and n else 0
    for t in range(T):
        run_copies_and_gathers(progs, bufs, t)
        sends = {}
        for r in range(P):
            for row in progs[r][progs[r][:, 0] == t]:
                if row[1] == 0:
                    _, _, peer, ring, b, off, cnt, _ = row
                    assert (r, peer, ring) not in sends
                    sends[(r, peer, ring)] = bufs[r][b][off:off + cnt].copy()
        for r in range(P):
            for row in progs[r][progs[r][:, 0] == t]:
                if row[1] == 1:
                    _, _, peer, ring, b, off, cnt, _ = row
                    data = sends.pop((peer, r, ring))
                    assert data.size == cnt
                    bufs[r][b][off:off + cnt] = data
        assert not sends, f'unmatched sends at tick {t}: {list(sends)}'
        for r in range(P):
            rows = progs[r][progs[r][:, 0] == t]
            for row in rows:
                if row[1] == 2:
                    _, _, _, _, b, off, cnt, soff = row
                    bufs[r][1][off:off + cnt] = oracle.sum2(dt, bufs[r][0][off:off + cnt],
                                                            bufs[r][2][soff:soff + cnt])
            apply_folds(oracle, dt, rows, bufs[r])
    return [b[1] for b in bufs]


def run_copies_and_gathers(progs, bufs, t):
    """A tick's device copies (kind 4: buffer 0 -> dst buffer) and its allgather (kind 11: rank
    q's block at (send buffer, offset) lands at recv offset + q * count on every rank), on host
    buffers bufs[r] = [in, out, staging], in the order the executor posts them."""
    P = len(progs)
    for r in range(P):
        for row in progs[r][(progs[r][:, 0] == t) & (progs[r][:, 1] == 4)]:
            _, _, _, _, b, off, cnt, soff = row
            bufs[r][b][off:off + cnt] = bufs[r][0][soff:soff + cnt]
    blocks = []
    for r in range(P):
        rows = progs[r][(progs[r][:, 0] == t) & (progs[r][:, 1] == 11)]
        if len(rows):
            _, _, sb, so, _, _, cnt, _ = rows[0]
            blocks.append(bufs[r][sb][so:so + cnt].copy())
    if blocks:
        assert len(blocks) == P, f'allgather at tick {t} not on every rank'
        for r in range(P):
            _, _, _, _, rb, ro, cnt, _ = progs[r][(progs[r][:, 0] == t) & (progs[r][:, 1] == 11)][0]
            for q in range(P):
                bufs[r][rb][ro + q * cnt:ro + (q + 1) * cnt] = blocks[q]


# General N-input fold rows of a program dump: kind -> (oracle total_bytes argument, output
# buffer). Order: None = left fold, 4096 = MPICH's pre-fold + pairwise tree (> 2048-byte
# messages), 0 = MPICH's binomial tree (<= 2048 bytes). Kinds 5-7 write the output buffer,
# 8-10 a partial sum into staging (fold chains / trees beyond 16 ranks).
GENERAL_FOLDS = {5: (None, 1), 6: (4096, 1), 7: (0, 1), 8: (None, 2), 9: (4096, 2), 10: (0, 2)}


def apply_folds(oracle, dt, rows, bufs):
    """Run one tick's N-input folds of one rank (rows of that tick) on bufs = [in, out, staging]:
    kind 3 (in + staged inputs, left fold) and the general fold steps (every input named), in
    the order the engine launches them."""
    folds = rows[rows[:, 1] == 3]
    if len(folds):
        nb = int(folds[0, 2])
        assert len(folds) == nb and list(folds[:, 3]) == list(range(nb))
        off, cnt = int(folds[0, 5]), int(folds[0, 6])
        ins = [bufs[0][off:off + cnt]] + [bufs[2][s:s + cnt] for s in folds[:, 7]]
        bufs[1][off:off + cnt] = oracle.fold(dt, ins)
    gen = rows[np.isin(rows[:, 1], list(GENERAL_FOLDS))]
    i = 0
    while i < len(gen):
        ni = int(gen[i, 2])
        step = gen[i:i + ni]
        assert len(step) == ni and list(step[:, 3]) == list(range(ni)) and len(set(step[:, 1])) == 1
        tb, ob = GENERAL_FOLDS[int(step[0, 1])]
        cnt, off = int(step[0, 6]), int(step[0, 7])
        ins = [bufs[int(b)][int(s):int(s) + cnt].copy() for b, s in zip(step[:, 4], step[:, 5])]
        bufs[ob][off:off + cnt] = oracle.fold(dt, ins) if tb is None else oracle.fold_ref_order(dt, ins, tb)
        i += ni


MPI_HOME = os.environ.get('MPI_HOME', '/opt/conda')
MPI_DRIVER = os.path.join(ROOT, 'oracle', 'build', 'mpi_allreduce_driver')


def live_mpich_available():
    return os.path.exists(MPI_DRIVER) and os.path.exists(os.path.join(MPI_HOME, 'bin', 'mpiexec'))


def live_mpich(xs, dt):
    """MPICH's own MPI_Allreduce(MPI_SUM) of the rank buffers xs (one process per rank, our
    oracle/mpi_allreduce_driver.c calling MPI as MPICommunicator.cc:14-28 does): rank 0's
    output; every rank's output must be identical. Test infrastructure only."""
    import subprocess
    import tempfile
    with tempfile.TemporaryDirectory() as d:
        for r, x in enumerate(xs):
            np.ascontiguousarray(x).tofile(os.path.join(d, f'in_{r}.bin'))
        env = dict(os.environ)
        env['LD_LIBRARY_PATH'] = os.path.join(MPI_HOME, 'lib') + ':' + env.get('LD_LIBRARY_PATH', '')
        subprocess.run([os.path.join(MPI_HOME, 'bin', 'mpiexec'), '-n', str(len(xs)), MPI_DRIVER, str(dt),
                        str(xs[0].size), d], check=True, env=env, timeout=120, capture_output=True)
        outs = [np.fromfile(os.path.join(d, f'out_{r}.bin'), dtype=xs[0].dtype) for r in range(len(xs))]
    assert all(o.tobytes() == outs[0].tobytes() for o in outs), 'MPICH ranks disagree'
    return outs[0]


def hip_runtime():
    """The HIP runtime torch and the engine already share, bound by soname with RTLD_NOLOAD (a
    second runtime loaded by file name would be handed torch's streams: tools/graph_probe.py),
    with the graph-capture entry points' signatures."""
    vp, ci, sz = ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t
    hip = ctypes.CDLL('libamdhip64.so.7', mode=os.RTLD_NOLOAD | os.RTLD_NOW)
    for name, res, args in (('hipStreamBeginCapture', ci, [vp, ci]),
                            ('hipStreamEndCapture', ci, [vp, ctypes.POINTER(vp)]),
                            ('hipGraphGetNodes', ci, [vp, vp, ctypes.POINTER(sz)]),
                            ('hipGraphGetEdges', ci, [vp, vp, vp, ctypes.POINTER(sz)]),
                            ('hipGraphInstantiate', ci, [ctypes.POINTER(vp), vp, vp, vp, sz]),
                            ('hipGraphLaunch', ci, [vp, vp]),
                            ('hipGraphExecDestroy', ci, [vp]),
                            ('hipGraphDestroy', ci, [vp])):
        f = getattr(hip, name)
        f.restype, f.argtypes = res, args
    return hip


GOLDEN_FULLSIZE = os.path.join(ROOT, 'tests', 'golden', 'golden_fullsize.json')


def fullsize_cases():
    """MPICH 3.3.2's full-size outputs, pinned by hash (tests/golden/make_golden.py --fullsize):
    [(name, P, n, sha256, {index: value})]."""
    import json
    with open(GOLDEN_FULLSIZE) as f:
        cases = json.load(f)['cases']
    return [(k, c['P'], c['n'], c['sha256'], {int(i): v for i, v in c['samples'].items()})
            for k, c in sorted(cases.items())]


def fullsize_inputs(P, n):
    """The full-size cases' rank inputs, regenerated from make_golden.py's seed rule
    (default_rng(1234 + 7919 * rank).standard_normal(n) as fp32)."""
    return [np.random.default_rng(1234 + 7919 * r).standard_normal(n).astype(np.float32) for r in range(P)]


def sha256(a):
    import hashlib
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def fp16_single_rounding_bound(P, y, mag):
    """|y - Σx| bound of an fp16 allreduce that folds all P inputs in fp32 and rounds ONCE (the
    direct schedule, reference_order 1: DESIGN §3): ulp16(y)/2 for the one rounding plus
    (P-1)·2^-24·Σ|x| for the fp32 fold. ulp16 is taken at the output's own binade (a sum just
    below a power of two can round up into the next one); subnormals have ulp 2^-24. (A ring that
    rounds at every hop would need (P-1)·2^-11·Σ|x|: 8192x looser, VERDICT r5 weak #1.)"""
    import torch
    a = y.double().abs()
    _, e = torch.frexp(a)  # a = m * 2^e, m in [0.5, 1)
    ulp = torch.where(a > 0, torch.exp2((e - 11).double()), torch.full_like(a, 2.0 ** -24)).clamp_min(2.0 ** -24)
    return ulp / 2 + (P - 1) * 2.0 ** -24 * mag
