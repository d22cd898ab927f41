"""Soak run of the N>1 engine on one GPU (measurement / robustness, not a test): P processes over
the test transport repeat the concurrency-heavy checks of tests/_mp_gpu_worker.py — keyed rounds
placed among concurrent direct collectives (random pacing), split communicators with their own
token rings, keyed fusion, the grouped allreduce — `rounds` times, to flush out rare ordering
races or hangs before a node runs the engine. Usage: python tools/soak_mp.py [P=4] [rounds=10]"""
import os
import socket
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, os.path.join(ROOT, 'tests'))
# the workers need the test transport: the testing build (the spawned processes inherit this)
os.environ.setdefault('ddl_lib', os.path.join(ROOT, 'experiment-distributed-deep-learning_amd', 'lib',
                                              'libddl_amd_testing.so'))


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


def main():
    import torch.multiprocessing as mp

    import _mp_gpu_worker as w
    P = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    only = os.environ.get('SOAK_CHECKS')
    per_round = only.split(',') if only else ['check_keyed_round_order', 'check_split_communicators_keyed',
                                              'check_keyed_fusion', 'check_allreduce_batch']
    names = (per_round + ['check_resources']) * rounds
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    t0 = time.time()
    procs = [ctx.Process(target=w.worker, args=(r, P, PORT, q, names)) for r in range(P)]
    for p in procs:
        p.start()
    res = {}
    try:
        for _ in range(P):
            rank, results = q.get(timeout=900)
            res[rank] = results
    finally:
        for p in procs:
            p.join(timeout=30)
            if p.is_alive():
                p.kill()
    ok = all(all(o for _, o, _ in r) for r in res.values()) and len(res) == P
    print(f'soak P={P} rounds={rounds}: {"ok" if ok else "FAILED"} in {time.time() - t0:.0f} s, '
          f'{sum(len(r) for r in res.values())} check runs')
    for rank, results in sorted(res.items()):
        for name, o, detail in results:
            if not o:
                print(rank, name, detail[-800:])
    sys.exit(0 if ok else 1)


PORT = _free_port()
if __name__ == '__main__':
    main()
