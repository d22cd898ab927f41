"""The N>1 product path with REAL multi-rank RCCL communicators on one GPU (VERDICT r5 missing #1).
P processes share the card; each gets a host id of its own (NCCL_HOSTID, _mp_gpu_worker.
rccl_sockets_env), so RCCL does not refuse them as duplicates of one device and connects them with
its socket network transport over loopback. The engine then runs exactly as on a node — ddl_init
builds the world with ncclCommInitRankConfig at size P, splits use ncclCommSplit across ranks, the
keyed data plane its private split, every schedule's sends and receives are RcclTransport pairs
between the processes, the tuner agrees through ncclAllReduce(MAX) — and only the wire (sockets,
not xGMI) differs. Every check of tests/_mp_gpu_worker.py runs: bit-exact vs the oracle / MPICH's
order / exact sums."""
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


# P processes of 4 hardware queues each, beside the test process's own, can oversubscribe the GPU's
# hardware queue slots; the scheduler then time-slices the queues and RCCL's spinning kernels crawl
# (r06 s13: the P = 5 worker silent for minutes inside the whole suite, 50 s alone). So the suite
# runs the whole worker at P <= 4 and single-communicator checks at P = 5, 8 with 2 queues per rank;
# DDL_TEST_RCCL_BIG=1 adds the whole worker at P = 5, 8 (run in sessions: profiles/r06/s8, s9).
BIG = os.environ.get('DDL_TEST_RCCL_BIG') == '1'


def _run(world, only=None, timeout=300.0, hw_queues=None):
    import torch.multiprocessing as mp

    import _mp_gpu_worker
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_mp_gpu_worker.worker, args=(r, world, port, q, only, 'rccl')) for r in range(world)]
    old = os.environ.get('DDL_MP_HW_QUEUES')
    if hw_queues:  # the children read it before HIP starts (rccl_sockets_env)
        os.environ['DDL_MP_HW_QUEUES'] = str(hw_queues)
    try:
        for p in procs:
            p.start()
    finally:
        if hw_queues:
            if old is None:
                os.environ.pop('DDL_MP_HW_QUEUES', None)
            else:
                os.environ['DDL_MP_HW_QUEUES'] = old
    res = {}
    try:
        for _ in range(world):
            rank, results = q.get(timeout=float(os.environ.get('DDL_MP_TIMEOUT', timeout)))
            res[rank] = results
    finally:
        for p in procs:
            p.join(timeout=20)
        for p in procs:  # only our own children, by handle
            if p.is_alive():
                p.kill()
                p.join(timeout=10)
    assert sorted(res) == list(range(world)), f'ranks reported: {sorted(res)}'
    for rank, results in sorted(res.items()):
        for name, ok, detail in results:
            assert ok, f'rank {rank} {name}:\n{detail}'
    return res


@pytest.mark.parametrize('world', [2, 3, 4] + ([5, 8] if BIG else []))
def test_engine_over_multirank_rccl(gpu, world):
    """Every check of the multi-process worker at P ranks over real RCCL communicators."""
    import _mp_gpu_worker
    res = _run(world)
    names = [n for n, _, _ in res[0]]
    assert names == [f.__name__ for f in _mp_gpu_worker.CHECKS], names


@pytest.mark.parametrize('world', [2, 3])
def test_queue_isolation_over_rccl(gpu, world, monkeypatch):
    """Config queue_isolation = 1 from ddl_init on (the worker sets it before the world exists):
    the world's keyed data plane at the greatest stream priority, splits at the least, read back;
    the world's keyed rounds beside a split's stay bit-exact vs MPICH's order."""
    monkeypatch.setenv('DDL_MP_QUEUE_ISOLATION', '1')  # spawned children inherit it
    names = ['check_split_communicators_keyed', 'check_queue_classes']
    res = _run(world, names, timeout=180)
    for rank, results in res.items():
        assert [n for n, _, _ in results] == names, results


@pytest.mark.parametrize('world', [2, 3])
def test_control_link_lost_mid_round_over_rccl(gpu, world):
    """ADVICE r3's fault case over real RCCL communicators: a control link lost after a member froze
    its user collectives for a keyed round stops every rank's handler; keyed requests complete with
    an error and direct collectives return one instead of hanging (check_control_link_lost)."""
    res = _run(world, ['check_control_link_lost'], timeout=120)
    for rank, results in res.items():
        assert [n for n, _, _ in results][:1] == ['check_control_link_lost'], results


def test_data_parallelism_example_over_two_rccl_ranks():
    """The reference's DP script on this surface (examples/data_parallelism.py) as two training
    processes over one real two-rank RCCL communicator, each loading the deployment library alone
    (no ddl_lib override): the data sharded, the lr scaled by the size and warmed up to it, the
    initial weights broadcast, every step's gradients averaged through keyed fused allreduces, the
    metrics averaged — and the loss falls."""
    import re
    import subprocess
    import sys

    import _mp_gpu_worker
    from conftest import ROOT
    port = _free_port()
    procs = []
    for r in range(2):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE='2', LOCAL_RANK='0', MASTER_ADDR='127.0.0.1',
                   MASTER_PORT=str(port), **_mp_gpu_worker.rccl_sockets_env(r, 2))
        env.pop('ddl_lib', None)
        procs.append(subprocess.Popen([sys.executable, os.path.join(ROOT, 'examples', 'data_parallelism.py'),
                                       '--epochs', '3', '--samples', '4096', '--warmup_epochs', '2', '--lr', '0.002'],
                                      env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True))
    outs = []
    try:
        for p in procs:
            outs.append(p.communicate(timeout=300))
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
                p.wait()
    for p, (out, err) in zip(procs, outs):
        assert p.returncode == 0, err[-3000:]
    out0 = outs[0][0]
    losses = [float(m) for m in re.findall(r'loss ([0-9.e+-]+)', out0)]
    lrs = [float(m) for m in re.findall(r'lr ([0-9.e+-]+)', out0)]
    assert len(losses) == 3 and losses[-1] < losses[0], out0
    assert lrs[1] == pytest.approx(2 * 0.002, rel=1e-6)  # warmed up to size x lr after 2 epochs
    assert 'finished gradual learning rate warmup' in out0


@pytest.mark.parametrize('world', [5, 8])
def test_full_size_hash_equals_mpich_over_multirank_rccl(gpu, world):
    """C3 (P = 8, 256 MiB fp32 per rank) and the P = 5 pre-fold at full size through real multi-rank
    RCCL communicators: every rank's output hashes to MPICH 3.3.2's (check_fullsize_mpich_hash)."""
    res = _run(world, ['check_fullsize_mpich_hash'], timeout=300, hw_queues=2)  # one communicator in use
    for rank, results in res.items():
        assert [n for n, _, _ in results][:1] == ['check_fullsize_mpich_hash'], results


@pytest.mark.parametrize('world', [2, 3])
def test_graph_capture_over_multirank_rccl(gpu, world):
    """hipGraph capture of the data plane with real RCCL kernels between processes, serial and DAG
    posting, three schedules, replayed on fresh inputs bit-exact (check_graph_capture)."""
    res = _run(world, ['check_graph_capture'], timeout=240)
    for rank, results in res.items():
        assert [n for n, _, _ in results][:1] == ['check_graph_capture'], results
