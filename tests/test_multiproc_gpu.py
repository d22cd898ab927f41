"""The N>1 product path on one GPU: P = 2, 3, 4, 5, 8 processes (5: the only P <= 8 where MPICH's
two summation orders differ) share the card and run the engine
end to end — world communicator, TCP token ring, keyed handler (negotiation, dtype groups,
fusion pipeline, cached ids), ring / direct / one-shot schedules, the collective autotuner,
broadcast / allgather, the host-resident pipeline and the scripts-level DP wrapper and
callbacks — checked against the oracle and exact sums (tests/_mp_gpu_worker.py). Only the
point-to-point groups differ from an RCCL run: they go through gloo on host copies
(ddl_init_test_transport), because RCCL refuses two ranks of one host on one device. The same
worker over real multi-rank RCCL (a host id per rank, RCCL's socket transport): test_multiproc_rccl_gpu.py."""
import os
import socket

import pytest

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize('world,pipelined', [(2, 1), (3, 1), (4, 1), (5, 1), (8, 1), (4, 0)])
def test_engine_multiprocess_on_one_gpu(gpu, world, pipelined, monkeypatch):
    """Every check at P ranks; keyed rounds pipelined (default) and, at P = 4, waited for one by
    one (pipeline_rounds = 0, the spawned workers read DDL_MP_PIPELINE_ROUNDS). The P = 8 case
    takes 40-100 s box to box (eight processes share one GPU and the box's CPU share; r04 saw
    ~100 s), so the wait for the ranks' results is 300 s (DDL_MP_TIMEOUT)."""
    import torch.multiprocessing as mp
    monkeypatch.setenv('DDL_MP_PIPELINE_ROUNDS', str(pipelined))

    import _mp_gpu_worker
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_mp_gpu_worker.worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    try:
        for _ in range(world):
            rank, results = q.get(timeout=float(os.environ.get('DDL_MP_TIMEOUT', 300)))
            res[rank] = results
    finally:
        for p in procs:
            p.join(timeout=20)
        for p in procs:  # only our own children, by handle
            if p.is_alive():
                p.kill()
                p.join(timeout=10)
    assert sorted(res) == list(range(world)), f'ranks reported: {sorted(res)}'
    names = [n for n, _, _ in res[0]]
    assert names and names[-1] == _mp_gpu_worker.CHECKS[-1].__name__ or any(not ok for _, ok, _ in res[0]), names
    for rank, results in sorted(res.items()):
        for name, ok, detail in results:
            assert ok, f'rank {rank} {name}:\n{detail}'


@pytest.mark.parametrize('world', [2, 3])
def test_control_link_lost_mid_round(gpu, world):
    """a control link lost after a member froze its user collectives for a keyed round
    stops every rank's handler; keyed requests complete with an error and direct collectives
    return one instead of hanging (tests/_mp_gpu_worker.py check_control_link_lost)."""
    import torch.multiprocessing as mp

    import _mp_gpu_worker
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_mp_gpu_worker.worker, args=(r, world, port, q, ['check_control_link_lost']))
             for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    try:
        for _ in range(world):
            rank, results = q.get(timeout=120)
            res[rank] = results
    finally:
        for p in procs:
            p.join(timeout=20)
        for p in procs:
            if p.is_alive():
                p.kill()
                p.join(timeout=10)
    assert sorted(res) == list(range(world)), f'ranks reported: {sorted(res)}'
    for rank, results in sorted(res.items()):
        assert [n for n, _, _ in results][:1] == ['check_control_link_lost'], results
        for name, ok, detail in results:
            assert ok, f'rank {rank} {name}:\n{detail}'
