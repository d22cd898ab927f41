"""Replay time of a captured P-rank allreduce posted as a single-stream DAG (capture_mode 2) vs
serially (capture_mode 0), one GPU (measurement). World 'local' moves the slices by
D2D copies, 'rccl' through the one-rank RCCL loopback. Prints one JSON line per case with the
graph's node / edge count and longest dependency chain.
    python tools/capture_overlap.py [world=local] [P=4]"""
import ctypes
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault('ddl_lib', os.path.join(ROOT, 'experiment-distributed-deep-learning_amd', 'lib', 'libddl_amd_testing.so'))  # the testing build (raw kernels, test transport)
sys.path.insert(0, os.path.join(ROOT, 'experiment-distributed-deep-learning_amd'))
sys.path.insert(0, os.path.join(ROOT, 'tests'))
from ddl.torch.cpp_backend import CPPBackend  # noqa: E402
from _helpers import hip_runtime  # noqa: E402
from test_graph_gpu import _graph_shape  # noqa: E402


def transitive_reduction(hip, g):
    """Removes every edge a -> b of g that another path a -> ... -> b implies."""
    vp = ctypes.c_void_p
    ne = ctypes.c_size_t(0)
    assert hip.hipGraphGetEdges(g, None, None, ctypes.byref(ne)) == 0
    src, dst = (vp * ne.value)(), (vp * ne.value)()
    assert hip.hipGraphGetEdges(g, src, dst, ctypes.byref(ne)) == 0
    succ = {}
    for a, b in zip(src, dst):
        succ.setdefault(a, set()).add(b)
    reach = {}

    def reachable(a):  # nodes reachable from a by a path of >= 1 edge
        if a not in reach:
            r = set()
            for b in succ.get(a, ()):
                r.add(b)
                r |= reachable(b)
            reach[a] = r
        return reach[a]
    sys.setrecursionlimit(100000)
    drop = [(a, b) for a in succ for b in succ[a] if any(b in reachable(c) for c in succ[a] if c != b)]
    if drop:
        fa, fb = (vp * len(drop))(*[a for a, _ in drop]), (vp * len(drop))(*[b for _, b in drop])
        assert hip.hipGraphRemoveDependencies(g, fa, fb, ctypes.c_size_t(len(drop))) == 0


def main(world='local', P=4):
    lib = CPPBackend.c_api()
    hip = hip_runtime()
    f = hip.hipGraphRemoveDependencies
    f.restype, f.argtypes = ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t]
    dev = torch.device('cuda', 0)
    torch.cuda.set_device(dev)
    if world == 'rccl':
        assert lib.ddl_rccl_loopback_init(0) == 0, lib.ddl_last_error()
    s = torch.cuda.Stream()
    st = ctypes.c_void_p(s.cuda_stream)
    for nbytes, slice_bytes in ((256 << 10, 16 << 10), (4 << 20, 128 << 10), (64 << 20, 2 << 20)):
        n = nbytes // 4
        ins = [torch.randn(n, device=dev) for _ in range(P)]
        outs = [torch.empty_like(t) for t in ins]
        send = (ctypes.c_void_p * P)(*[t.data_ptr() for t in ins])
        recv = (ctypes.c_void_p * P)(*[t.data_ptr() for t in outs])

        def call():
            if world == 'local':
                return lib.ddl_local_ring_allreduce(P, send, recv, n, 1, 0, s.cuda_stream)
            return lib.ddl_rccl_loopback_allreduce(P, send, recv, n, 1, s.cuda_stream)

        for k, v in (('algo', 1), ('reference_order', 1), ('tune', 0), ('slice_bytes', slice_bytes)):
            assert lib.ddl_set_config(k.encode(), v) == 0
        eager = 1e9
        for _ in range(3):  # eager: the same program on the forked streams, launched from the host
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(10):
                assert call() == 0
            torch.cuda.synchronize()
            eager = min(eager, (time.perf_counter() - t0) / 10)
        print(json.dumps({'world': world, 'P': P, 'bytes_per_rank': nbytes, 'slice_bytes': slice_bytes,
                          'eager_us': round(eager * 1e6, 1)}), flush=True)
        for mode in (0, 2, 3):  # 3: the DAG with its transitively implied edges removed before instantiation
            for k, v in (('algo', 1), ('reference_order', 1), ('tune', 0), ('slice_bytes', slice_bytes),
                         ('capture_mode', min(mode, 2))):
                assert lib.ddl_set_config(k.encode(), v) == 0
            assert call() == 0, lib.ddl_last_error()
            torch.cuda.synchronize()
            assert hip.hipStreamBeginCapture(st, 0) == 0
            rc = call()
            g = ctypes.c_void_p()
            assert hip.hipStreamEndCapture(st, ctypes.byref(g)) == 0 and rc == 0
            if mode == 3:
                transitive_reduction(hip, g)
            nodes, edges, chain = _graph_shape(hip, g)
            x = ctypes.c_void_p()
            assert hip.hipGraphInstantiate(ctypes.byref(x), g, None, None, ctypes.c_size_t(0)) == 0
            reps = 20 if nbytes < (16 << 20) else 5
            best = 1e9
            for _ in range(3):
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for _ in range(reps):
                    assert hip.hipGraphLaunch(x, st) == 0
                torch.cuda.synchronize()
                best = min(best, (time.perf_counter() - t0) / reps)
            hip.hipGraphExecDestroy(x)
            hip.hipGraphDestroy(g)
            print(json.dumps({'world': world, 'P': P, 'bytes_per_rank': nbytes, 'slice_bytes': slice_bytes,
                              'capture_mode': ('serial', None, 'dag', 'dag_reduced')[mode], 'nodes': nodes, 'edges': edges,
                              'longest_chain': chain, 'replay_us': round(best * 1e6, 1)}), flush=True)
    if world == 'rccl':
        assert lib.ddl_rccl_loopback_finalize() == 0


if __name__ == '__main__':
    main(sys.argv[1] if len(sys.argv) > 1 else 'local', int(sys.argv[2]) if len(sys.argv) > 2 else 4)
