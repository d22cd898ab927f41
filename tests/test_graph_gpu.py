"""The data plane inside hipGraphs (torch.cuda.graph = hipStreamBeginCapture on the caller's
stream): one replay of a captured training step runs the engine's kernels and RCCL groups with no
host work per call — the small-bucket lever the host launch rate sets.

The engine is graph-safe by construction (executor.cpp `stream_capturing`): under capture it
enqueues only stream work — serially on the captured stream by default (capture_mode 0), or as a
single-stream DAG (capture_mode 2: every op on the captured stream, its dependencies set from its
logical comm / compute stream, so the graph keeps the recv / reduce / send overlap) — takes the size class's tuned
schedule or the configured one without tuning, and
refuses — loudly, before enqueueing anything — to grow its staging buffer or to capture a
transport that synchronises the host. Warm up once outside the capture, as for any captured
workload.

Bar: every replay bit-exact vs the oracle on fresh inputs written into the captured buffers —
MPICH's order (ddlo_fold_ref_order) for the allreduce over P virtual ranks whose moves go through
a real RCCL communicator (ddl_rccl_loopback_*), the restatement of MPI_SUM for the reduce kernel."""
import ctypes

import numpy as np
import pytest
import torch

from _helpers import DT_DOUBLE, DT_FLOAT, DT_INT32, NAME, config, hip_runtime, random_input

pytestmark = pytest.mark.gpu


def _t(x, dev):
    return torch.from_numpy(np.ascontiguousarray(x)).to(dev)


def test_reduce_kernel_graph_replay(lib, oracle, gpu):
    """K reduce launches captured into one graph; each replay on new data equals acc + in."""
    n, K = 100_003, 6
    s = torch.cuda.Stream()
    accs = [torch.empty(n, device=gpu) for _ in range(K)]
    ins = [torch.empty(n, device=gpu) for _ in range(K)]
    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(s):
        for a, b in zip(accs, ins):  # warm-up outside the capture
            assert lib.ddl_reduce_local(a.data_ptr(), b.data_ptr(), n, DT_FLOAT, s.cuda_stream) == 0
    torch.cuda.synchronize()
    with torch.cuda.graph(g, stream=s):
        for a, b in zip(accs, ins):
            assert lib.ddl_reduce_local(a.data_ptr(), b.data_ptr(), n, DT_FLOAT, s.cuda_stream) == 0, \
                lib.ddl_last_error()
    for rep in range(3):
        xa = [random_input(DT_FLOAT, n, 11 + rep * 100 + k) for k in range(K)]
        xb = [random_input(DT_FLOAT, n, 12 + rep * 100 + k) for k in range(K)]
        for k in range(K):
            accs[k].copy_(_t(xa[k], gpu))
            ins[k].copy_(_t(xb[k], gpu))
        g.replay()
        torch.cuda.synchronize()
        for k in range(K):
            assert accs[k].cpu().numpy().tobytes() == oracle.sum2(DT_FLOAT, xa[k], xb[k]).tobytes(), (rep, k)


def test_world_allreduce_graph_replay(lib, gpu):
    """The world communicator (one process: out = in) captured and replayed."""
    from ddl.torch.communicator import Communicator
    comm = Communicator.world()
    n = 4097
    s = torch.cuda.Stream()
    a = torch.empty(n, device=gpu)
    b = torch.empty(n, device=gpu)
    with torch.cuda.stream(s):
        assert lib.ddl_allreduce(comm.id, a.data_ptr(), b.data_ptr(), n, DT_FLOAT, 0, s.cuda_stream) == 0
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        assert lib.ddl_allreduce(comm.id, a.data_ptr(), b.data_ptr(), n, DT_FLOAT, 0, s.cuda_stream) == 0
    for rep in range(2):
        a.copy_(torch.randn(n, device=gpu))
        g.replay()
        torch.cuda.synchronize()
        assert torch.equal(a, b)


@pytest.fixture(scope='module')
def loop(lib, gpu):
    st = lib.ddl_rccl_loopback_init(0)
    assert st == 0, lib.ddl_last_error()
    yield lib
    assert lib.ddl_rccl_loopback_finalize() == 0, lib.ddl_last_error()


def _loop_allreduce(lib, ins, outs, n, dt, stream):
    P = len(ins)
    send = (ctypes.c_void_p * P)(*[t.data_ptr() for t in ins])
    recv = (ctypes.c_void_p * P)(*[t.data_ptr() for t in outs])
    return lib.ddl_rccl_loopback_allreduce(P, send, recv, n, dt, stream)


TORCH_DT = {DT_FLOAT: torch.float32, DT_DOUBLE: torch.float64, DT_INT32: torch.int32}


@pytest.mark.parametrize('mode', [2, 0], ids=['dag', 'serial'])
@pytest.mark.parametrize('P', [3, 5, 8])
@pytest.mark.parametrize('dt', [DT_FLOAT, DT_DOUBLE, DT_INT32], ids=lambda d: NAME[d])
@pytest.mark.parametrize('algo', [1, 2, 3, 4])
def test_rccl_allreduce_graph_replay(loop, oracle, gpu, P, dt, algo, mode):
    """P virtual ranks' allreduce, moves through RCCL, captured once and replayed on fresh
    inputs: every rank equals MPICH's order bit for bit on both sides of the 2048-byte switch,
    out of place and in place; posted as a single-stream DAG and serially (the default)."""
    lib = loop
    s = torch.cuda.Stream()
    with config(lib, algo=algo, reference_order=1, tune=0, slice_bytes=64 << 10, capture_mode=mode):
        for n in (300, 70_001, 128 * 840):  # 128 * 840: equal chunks (direct-gather's allgather)
            for in_place in (False, True):
                ins = [torch.zeros(n, dtype=TORCH_DT[dt], device=gpu) for _ in range(P)]
                outs = ins if in_place else [torch.empty_like(t) for t in ins]
                with torch.cuda.stream(s):  # warm-up: sizes staging and events
                    assert _loop_allreduce(lib, ins, outs, n, dt, s.cuda_stream) == 0, lib.ddl_last_error()
                torch.cuda.synchronize()
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g, stream=s):
                    assert _loop_allreduce(lib, ins, outs, n, dt, s.cuda_stream) == 0, lib.ddl_last_error()
                for rep in range(2):
                    xs = [random_input(dt, n, 7 + 31 * rep + 7919 * r + n) for r in range(P)]
                    for r in range(P):
                        ins[r].copy_(_t(xs[r], gpu))
                    g.replay()
                    torch.cuda.synchronize()
                    want = oracle.fold_ref_order(dt, xs).tobytes()
                    for r in range(P):
                        assert outs[r].cpu().numpy().tobytes() == want, (n, in_place, rep, r)
                del g


def test_capture_refuses_to_grow_staging(loop, gpu):
    """A first call inside a capture would have to allocate staging: refused with a status and a
    message, nothing enqueued, the capture still ends cleanly."""
    lib = loop
    P, n = 4, 3_000_001  # larger than every earlier call: the staging must grow
    s = torch.cuda.Stream()
    ins = [torch.zeros(n, device=gpu) for _ in range(P)]
    outs = [torch.empty_like(t) for t in ins]
    g = torch.cuda.CUDAGraph()
    with config(lib, algo=1, reference_order=1, tune=0, slice_bytes=64 << 10):
        small = [t[:10] for t in ins], [t[:10] for t in outs]
        with torch.cuda.stream(s):  # the 4-rank world exists (streams, events) before the capture
            assert _loop_allreduce(lib, small[0], small[1], 10, DT_FLOAT, s.cuda_stream) == 0
        torch.cuda.synchronize()
        with torch.cuda.graph(g, stream=s):
            st = _loop_allreduce(lib, ins, outs, n, DT_FLOAT, s.cuda_stream)
        assert st != 0
        assert 'capture' in lib.ddl_last_error().decode()
        # outside the capture the same call works
        with torch.cuda.stream(s):
            assert _loop_allreduce(lib, ins, outs, n, DT_FLOAT, s.cuda_stream) == 0, lib.ddl_last_error()
        torch.cuda.synchronize()


def test_captured_staging_survives_later_growth(loop, oracle, gpu):
    """a captured graph keeps the address of each virtual rank's staging buffer. A
    later eager allreduce with a larger bucket must not free it (the engine retires it instead):
    replaying the graph afterwards still equals MPICH's order bit for bit."""
    lib = loop
    P, n_small, n_big = 6, 70_001, 4_000_003
    s = torch.cuda.Stream()
    with config(lib, algo=1, reference_order=1, tune=0, slice_bytes=64 << 10):
        ins = [torch.zeros(n_small, device=gpu) for _ in range(P)]
        outs = [torch.empty_like(t) for t in ins]
        with torch.cuda.stream(s):
            assert _loop_allreduce(lib, ins, outs, n_small, DT_FLOAT, s.cuda_stream) == 0, lib.ddl_last_error()
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            assert _loop_allreduce(lib, ins, outs, n_small, DT_FLOAT, s.cuda_stream) == 0, lib.ddl_last_error()
        big_in = [torch.randn(n_big, device=gpu) for _ in range(P)]
        big_out = [torch.empty_like(t) for t in big_in]
        with torch.cuda.stream(s):  # grows every rank's staging
            assert _loop_allreduce(lib, big_in, big_out, n_big, DT_FLOAT, s.cuda_stream) == 0, lib.ddl_last_error()
        torch.cuda.synchronize()
        # memory freed by a growth would be handed out again: fill fresh allocations with garbage
        junk = [torch.full((n_big,), float('nan'), device=gpu) for _ in range(P)]
        torch.cuda.synchronize()
        for rep in range(2):
            xs = [random_input(DT_FLOAT, n_small, 101 + 31 * rep + 7919 * r) for r in range(P)]
            for r in range(P):
                ins[r].copy_(_t(xs[r], gpu))
            g.replay()
            torch.cuda.synchronize()
            want = oracle.fold_ref_order(DT_FLOAT, xs).tobytes()
            for r in range(P):
                assert outs[r].cpu().numpy().tobytes() == want, (rep, r)
        del g, junk


def _graph_shape(hip, g):
    """(nodes, edges, longest dependency chain in nodes) of a hipGraph."""
    vp = ctypes.c_void_p
    nn, ne = ctypes.c_size_t(0), ctypes.c_size_t(0)
    assert hip.hipGraphGetNodes(g, None, ctypes.byref(nn)) == 0
    nodes = (vp * nn.value)()
    assert hip.hipGraphGetNodes(g, nodes, ctypes.byref(nn)) == 0
    assert hip.hipGraphGetEdges(g, None, None, ctypes.byref(ne)) == 0
    src, dst = (vp * max(1, ne.value))(), (vp * max(1, ne.value))()
    if ne.value:
        assert hip.hipGraphGetEdges(g, src, dst, ctypes.byref(ne)) == 0
    succ, indeg = {}, {n: 0 for n in nodes}
    for a, b in zip(src[:ne.value], dst[:ne.value]):
        succ.setdefault(a, []).append(b)
        indeg[b] += 1
    depth = {n: 1 for n in nodes}
    ready = [n for n in nodes if indeg[n] == 0]
    while ready:  # longest path by topological order
        a = ready.pop()
        for b in succ.get(a, []):
            depth[b] = max(depth[b], depth[a] + 1)
            indeg[b] -= 1
            if indeg[b] == 0:
                ready.append(b)
    return nn.value, ne.value, max(depth.values()) if depth else 0


@pytest.mark.parametrize('world', ['local', 'rccl'])
def test_dag_capture_keeps_the_overlap(loop, oracle, gpu, world):
    """captured as a single-stream DAG (capture_mode 2) the direct program of P = 4
    ranks with 8 slices per chunk is a graph whose longest dependency chain is much shorter than
    its node count — the ranks' moves, folds and allgathers stay concurrent — while the serial
    capture (capture_mode 0) is one chain; both replay bit-exact vs MPICH's order. The capture goes
    through hipStreamBeginCapture / hipStreamEndCapture on the runtime torch loaded."""
    lib = loop
    hip = hip_runtime()
    P, n = 4, 4 * 8 * 4096  # 8 slices of 16 KiB per chunk
    s = torch.cuda.Stream()
    ins = [torch.zeros(n, device=gpu) for _ in range(P)]
    outs = [torch.empty_like(t) for t in ins]
    send = (ctypes.c_void_p * P)(*[t.data_ptr() for t in ins])
    recv = (ctypes.c_void_p * P)(*[t.data_ptr() for t in outs])

    def call():
        if world == 'local':
            return lib.ddl_local_ring_allreduce(P, send, recv, n, DT_FLOAT, 0, s.cuda_stream)
        return lib.ddl_rccl_loopback_allreduce(P, send, recv, n, DT_FLOAT, s.cuda_stream)

    shapes = {}
    for mode in (2, 0):
        with config(lib, algo=1, reference_order=1, tune=0, slice_bytes=16 << 10, capture_mode=mode):
            assert call() == 0, lib.ddl_last_error()  # warm-up
            torch.cuda.synchronize()
            st = ctypes.c_void_p(s.cuda_stream)
            assert hip.hipStreamBeginCapture(st, 0) == 0
            rc = call()
            g = ctypes.c_void_p()
            assert hip.hipStreamEndCapture(st, ctypes.byref(g)) == 0
            assert rc == 0, lib.ddl_last_error()
            shapes[mode] = _graph_shape(hip, g)
            x = ctypes.c_void_p()
            assert hip.hipGraphInstantiate(ctypes.byref(x), g, None, None, ctypes.c_size_t(0)) == 0
            for rep in range(2):
                xs = [random_input(DT_FLOAT, n, 300 + 31 * rep + 7919 * r + mode) for r in range(P)]
                for r in range(P):
                    ins[r].copy_(_t(xs[r], gpu))
                torch.cuda.synchronize()
                assert hip.hipGraphLaunch(x, st) == 0
                torch.cuda.synchronize()
                want = oracle.fold_ref_order(DT_FLOAT, xs).tobytes()
                for r in range(P):
                    assert outs[r].cpu().numpy().tobytes() == want, (mode, rep, r)
            assert hip.hipGraphExecDestroy(x) == 0
            assert hip.hipGraphDestroy(g) == 0
    nodes, edges, chain = shapes[2]
    s_nodes, s_edges, s_chain = shapes[0]
    assert s_chain > chain, shapes
    if world == 'local':  # only the engine's own nodes: the serial capture is exactly one chain
        assert s_chain == s_nodes and nodes >= 8 and chain * 2 <= nodes, shapes
    else:  # RCCL adds nodes of its own per group; the folds of every rank still run beside them
        assert nodes >= 8 and chain * 4 <= nodes * 3, shapes


@pytest.mark.parametrize('P', [3, 8])
def test_dag_capture_broadcast_allgatherv(loop, oracle, gpu, P):
    """Broadcast and allgatherv of P virtual ranks over the RCCL loopback captured as DAGs and
    replayed: equal to MPI_Bcast / MPI_Allgatherv's restatements on fresh inputs."""
    lib = loop
    s = torch.cuda.Stream()
    n = 50_003
    bufs = [torch.zeros(n, device=gpu) for _ in range(P)]
    arr = (ctypes.c_void_p * P)(*[b.data_ptr() for b in bufs])
    counts = [700 * (q + 1) + q for q in range(P)]
    displs = [int(d) for d in np.cumsum([0] + counts[:-1])]
    sends = [torch.zeros(c, dtype=torch.int32, device=gpu) for c in counts]
    recvs = [torch.zeros(sum(counts), dtype=torch.int32, device=gpu) for _ in range(P)]
    Sz = ctypes.c_size_t * P
    sa = (ctypes.c_void_p * P)(*[d.data_ptr() for d in sends])
    ra = (ctypes.c_void_p * P)(*[r.data_ptr() for r in recvs])
    root = P - 1
    with config(lib, capture_mode=2, tune=0, slice_bytes=64 << 10):
        def call():
            assert lib.ddl_rccl_loopback_broadcast(P, root, arr, n, DT_FLOAT, s.cuda_stream) == 0, lib.ddl_last_error()
            assert lib.ddl_rccl_loopback_allgatherv(P, sa, ra, Sz(*counts), Sz(*displs), DT_INT32,
                                                    s.cuda_stream) == 0, lib.ddl_last_error()
        with torch.cuda.stream(s):
            call()
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            call()
        for rep in range(2):
            xs = [random_input(DT_FLOAT, n, 900 + rep * 10 + q) for q in range(P)]
            ys = [random_input(DT_INT32, c, 950 + rep * 10 + q) for q, c in enumerate(counts)]
            for q in range(P):
                bufs[q].copy_(_t(xs[q], gpu))
                sends[q].copy_(_t(ys[q], gpu))
            g.replay()
            torch.cuda.synchronize()
            for b, w in zip(bufs, oracle.broadcast(DT_FLOAT, xs, root)):
                assert b.cpu().numpy().tobytes() == w.tobytes(), rep
            want = oracle.allgatherv(DT_INT32, ys, displs).tobytes()
            for r in recvs:
                assert r.cpu().numpy().tobytes() == want, rep
        del g
