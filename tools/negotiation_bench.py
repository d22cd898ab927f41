"""Token-ring negotiation latency (host only): P processes on loopback TCP run rounds of
ddl_control_negotiate with the same 4096 gradient keys (the C5 / training-step case). Round 1
ships the ids as strings; later rounds ship them as indices into the shared id table.

    python tools/negotiation_bench.py [P ...]        (NEG_KEYS=1 NEG_ROUNDS=200: one-key rounds)
"""
import ctypes
import json
import os
import sys
import time

import multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault('ddl_lib', os.path.join(ROOT, 'experiment-distributed-deep-learning_amd', 'lib', 'libddl_amd_testing.so'))  # the testing build (raw kernels, test transport)
sys.path.insert(0, os.path.join(ROOT, 'experiment-distributed-deep-learning_amd'))

KEYS = [f'grad_{i:05d}' for i in range(int(os.environ.get('NEG_KEYS', 4096)))]
ROUNDS = int(os.environ.get('NEG_ROUNDS', 20))


def worker(rank, world, eps_q, go_q, out_q):
    from ddl.torch.cpp_backend import CPPBackend
    lib = CPPBackend.c_api()
    ep = ctypes.create_string_buffer(256)
    assert lib.ddl_control_listen(ep, 256) == 0
    eps_q.put((rank, ep.value.decode()))
    assert lib.ddl_control_connect_ranked(rank, world, go_q.get().encode()) == 0, lib.ddl_last_error()
    msg = '\n'.join(KEYS).encode()
    out = ctypes.create_string_buffer(1 << 17)
    times = []
    for _ in range(ROUNDS):
        t0 = time.perf_counter()
        assert lib.ddl_control_negotiate(msg, out, len(out)) == 0, lib.ddl_last_error()
        times.append(time.perf_counter() - t0)
    assert out.value.decode().count('\n') == len(KEYS)
    out_q.put((rank, times))


def run(world):
    ctx = mp.get_context('spawn')
    eps_q, out_q = ctx.Queue(), ctx.Queue()
    go = [ctx.Queue() for _ in range(world)]
    procs = [ctx.Process(target=worker, args=(r, world, eps_q, go[r], out_q)) for r in range(world)]
    for p in procs:
        p.start()
    eps = dict(eps_q.get(timeout=60) for _ in range(world))
    for q in go:
        q.put(';'.join(eps[r] for r in range(world)))
    res = dict(out_q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=30)
    t0 = res[0]
    return {'P': world, 'keys': len(KEYS), 'string_round_ms': round(t0[0] * 1e3, 3),
            'cached_round_ms_median': round(sorted(t0[1:])[len(t0[1:]) // 2] * 1e3, 3)}


if __name__ == '__main__':
    sizes = [int(a) for a in sys.argv[1:]] or [2, 4, 8]
    print(json.dumps({'cpus': os.cpu_count(), 'results': [run(P) for P in sizes]}))
