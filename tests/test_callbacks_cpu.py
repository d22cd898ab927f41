"""LearningRateSchedule / LearningRateWarmup (mirrors of the reference's Keras callbacks,
src/py/ddl/tensorflow/keras/parallelism/data/lr_warm_up_callback.py:6-124) against their formula:

    lr(epoch e, batch b) = initial_lr / size * ((e + (b + 1) / steps) * (size - 1) / warmup + 1)

for e < warmup; torch SGD's momentum left alone (its velocity does not hold the lr),
and with the correction forced (an optimizer keeping lr-scaled velocity, as Keras' SGD) the momentum
scaled by new_lr / old_lr during the batch and restored after it; the
lr left at initial_lr once the warm-up ends, and the closing message printed on rank 0 only. The
callbacks communicate nothing; they read the communicator's size and rank. Sizes 1, 2 and 8: in one
process with a stand-in communicator, and as gloo process groups whose ranks compare traces."""
import contextlib
import io
import os
import socket
import sys

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

HERE = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(os.path.dirname(HERE), 'experiment-distributed-deep-learning_amd')


class _Comm:
    def __init__(self, rank, size):
        self.rank, self.size = rank, size


def _expected(initial, size, warmup, steps, e, b):
    return initial / size * ((e + (b + 1) / steps) * (size - 1) / warmup + 1)


def _train(comm, epochs=3, steps=4, warmup=2, lr=0.4, momentum=0.9, verbose=1, correction=None):
    """A Keras-shaped loop over an SGD optimizer with two parameter groups; returns, per batch,
    (lr of each group during the batch, momentum during the batch, momentum after it), the logs'
    lr per epoch and what was printed."""
    from ddl.torch.parallelism.data import LearningRateWarmup
    w1, w2 = torch.nn.Parameter(torch.ones(3)), torch.nn.Parameter(torch.ones(2))
    opt = torch.optim.SGD([{'params': [w1]}, {'params': [w2], 'lr': lr / 2}], lr=lr, momentum=momentum)
    cb = LearningRateWarmup(opt, warmup_epochs=warmup, steps_per_epoch=steps, verbose=verbose, communicator=comm,
                            momentum_correction=correction)
    trace, logs_lr = [], []
    buf = io.StringIO()
    with contextlib.redirect_stdout(buf):
        cb.on_train_begin()
        for e in range(epochs):
            cb.on_epoch_begin(e)
            for b in range(steps):
                cb.on_batch_begin(b)
                during = ([g['lr'] for g in opt.param_groups], opt.param_groups[0]['momentum'])
                opt.zero_grad()
                (w1.sum() + w2.sum()).backward()
                opt.step()
                cb.on_batch_end(b)
                trace.append((during[0], during[1], opt.param_groups[0]['momentum']))
            logs = cb.on_epoch_end(e, {})
            logs_lr.append(logs['lr'])
    return trace, logs_lr, buf.getvalue()


def _check_trace(trace, logs_lr, printed, size, rank, epochs=3, steps=4, warmup=2, lr=0.4, momentum=0.9,
                 corrected=False):
    prev = [lr, lr / 2]
    for i, (lrs, m_during, m_after) in enumerate(trace):
        e, b = divmod(i, steps)
        if e < warmup:
            want = [_expected(lr, size, warmup, steps, e, b), _expected(lr / 2, size, warmup, steps, e, b)]
            assert lrs == pytest.approx(want, rel=1e-12), (e, b)
            if corrected:
                assert m_during == pytest.approx(momentum * want[0] / prev[0], rel=1e-12), (e, b)
            else:  # torch SGD: lr outside the velocity, nothing to correct
                assert m_during == momentum, (e, b)
        else:  # after the warm-up the lr stays where the last warm-up batch left it: initial_lr
            want = prev
            assert lrs == pytest.approx([lr, lr / 2], rel=1e-12), (e, b)
            assert m_during == momentum
        assert m_after == momentum  # restored after every batch
        prev = lrs
    assert logs_lr[warmup - 1] == pytest.approx(lr, rel=1e-12)
    assert ('finished gradual learning rate warmup' in printed) == (rank == 0)


@pytest.mark.parametrize('size', [1, 2, 8])
@pytest.mark.parametrize('rank', [0, 1])
def test_warmup_formula_in_process(size, rank):
    if rank >= size:
        pytest.skip('no such rank')
    sys.path.insert(0, PKG)
    trace, logs_lr, printed = _train(_Comm(rank, size))
    _check_trace(trace, logs_lr, printed, size, rank)


@pytest.mark.parametrize('size', [2, 8])
def test_momentum_correction_only_for_lr_scaled_velocity(size):
    """Default: torch.optim.SGD gets no momentum rescale (its first warm-up batch would otherwise
    drop momentum to about m / size). An optimizer declaring lr_scaled_velocity gets the
    reference's correction automatically; momentum_correction=True forces it."""
    sys.path.insert(0, PKG)
    from ddl.torch.parallelism.data import LearningRateWarmup
    trace, logs_lr, printed = _train(_Comm(0, size), correction=True)
    _check_trace(trace, logs_lr, printed, size, 0, corrected=True)
    w = torch.nn.Parameter(torch.ones(2))
    opt = torch.optim.SGD([w], lr=0.4, momentum=0.9)
    assert not LearningRateWarmup(opt, steps_per_epoch=4, communicator=_Comm(0, size)).momentum_correction
    opt.lr_scaled_velocity = True
    assert LearningRateWarmup(opt, steps_per_epoch=4, communicator=_Comm(0, size)).momentum_correction
    assert not LearningRateWarmup(opt, steps_per_epoch=4, communicator=_Comm(0, size),
                                  momentum_correction=False).momentum_correction


def test_schedule_staircase_constant_multiplier_and_autodetect():
    sys.path.insert(0, PKG)
    from ddl.torch.parallelism.data import LearningRateSchedule
    w = torch.nn.Parameter(torch.ones(2))
    opt = torch.optim.SGD([w], lr=1.0)  # no momentum: nothing to correct
    cb = LearningRateSchedule(opt, 0.5, start_epoch=1, end_epoch=3, staircase=False)
    assert cb.staircase  # a constant multiplier forces the staircase (reference :24-26)
    cb.on_train_begin()
    seen = []
    for e in range(4):
        cb.on_epoch_begin(e)
        for b in range(3):
            cb.on_batch_begin(b)
            seen.append(opt.param_groups[0]['lr'])
            cb.on_batch_end(b)
    assert seen == [1.0] * 3 + [0.5] * 9  # set at epoch 1's first batch, then left alone
    cb2 = LearningRateSchedule(opt, lambda e: e, staircase=False)
    with pytest.raises(ValueError, match='steps_per_epoch'):
        cb2.on_train_begin()
    cb3 = LearningRateSchedule(opt, lambda e: e, staircase=False)
    cb3.on_train_begin(params={'samples': 100, 'batch_size': 32})
    assert cb3.steps_per_epoch == 3


def _port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, size, port, q):
    try:
        sys.path.insert(0, PKG)
        dist.init_process_group('gloo', init_method=f'tcp://127.0.0.1:{port}', rank=rank, world_size=size)
        comm = _Comm(dist.get_rank(), dist.get_world_size())
        trace, logs_lr, printed = _train(comm)
        everyone = [None] * size
        dist.all_gather_object(everyone, (trace, logs_lr, 'finished gradual' in printed))
        if rank == 0:
            for r, (t, l, p) in enumerate(everyone):
                _check_trace(t, l, 'finished gradual learning rate warmup' if p else '', size, r)
                assert t == everyone[0][0]  # every rank the same schedule
        dist.destroy_process_group()
        q.put((rank, True, ''))
    except Exception as e:  # report instead of hanging the parent
        q.put((rank, False, repr(e)))


@pytest.mark.parametrize('size', [2, 8])
def test_warmup_over_gloo(size):
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_worker, args=(r, size, port, q)) for r in range(size)]
    for p in procs:
        p.start()
    res = [q.get(timeout=180) for _ in procs]
    for p in procs:
        p.join(30)
    assert all(ok for _, ok, _ in res), res
