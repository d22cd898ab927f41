"""Full-size parity against MPICH itself (VERDICT r5 next #1 / missing #3): C3 (P = 8, one 256 MiB
fp32 bucket per rank) and the non-power-of-two pre-fold at that size (P = 5, 7). The inputs are
regenerated here from make_golden.py's seed rule; MPICH 3.3.2's output is pinned by the sha256 in
tests/golden/golden_fullsize.json (what MPI_Allreduce returned in MPICommunicator.cc:14-28's call,
run in the build container). Every rank's output must hash to it, through

* the RCCL loopback (ddl_rccl_loopback_allreduce: P virtual ranks, the engine's RcclTransport on a
  real RCCL communicator), the default schedule and order, tuner off, out of place; and
* the asynchronous thread world with its pairs moved by RCCL (ddl_testing_thread_transport(1):
  P threads each driving RingExecutor::run_, what ddl_allreduce runs at N > 1), default schedule.

The schedule that runs is the library default (`algo` untouched): the direct schedule at P > 2
under reference_order 1."""
import ctypes

import numpy as np
import pytest
import torch

from _helpers import DT_FLOAT, config, fullsize_cases, fullsize_inputs, sha256

pytestmark = pytest.mark.gpu
CASES = fullsize_cases()


@pytest.fixture(scope='module')
def loop(lib, gpu):
    assert lib.ddl_rccl_loopback_init(0) == 0, lib.ddl_last_error()
    yield lib
    assert lib.ddl_rccl_loopback_finalize() == 0, lib.ddl_last_error()


def _ptrs(ts):
    return (ctypes.c_void_p * len(ts))(*[t.data_ptr() for t in ts])


def _check(outs, digest, samples, what):
    for r, o in enumerate(outs):
        y = o.cpu().numpy()
        bad = [i for i, v in samples.items() if float(y[i]) != v]
        assert not bad, (what, r, bad[:4])
        assert sha256(y) == digest, (what, r)


def _loopback(lib, ins, outs, n):
    st = lib.ddl_rccl_loopback_allreduce(len(ins), _ptrs(ins), _ptrs(outs), n, DT_FLOAT,
                                         torch.cuda.current_stream().cuda_stream)
    assert st == 0, lib.ddl_last_error()


def _thread_world_rccl(lib, ins, outs, n):
    before = ctypes.c_longlong(-1)
    assert lib.ddl_testing_thread_transport(1, ctypes.byref(before)) == 0, lib.ddl_last_error()
    try:
        st = lib.ddl_testing_thread_allreduce(len(ins), _ptrs(ins), _ptrs(outs), n, DT_FLOAT,
                                              torch.cuda.current_stream().cuda_stream)
        assert st == 0, lib.ddl_last_error()
        torch.cuda.synchronize()
        after = ctypes.c_longlong(-1)
        assert lib.ddl_testing_thread_transport(1, ctypes.byref(after)) == 0
        assert after.value > before.value, 'no send / receive pair went through RCCL'
    finally:
        assert lib.ddl_testing_thread_transport(0, None) == 0


@pytest.mark.parametrize('case', [c[0] for c in CASES])
@pytest.mark.parametrize('path', ['rccl_loopback', 'thread_world_rccl'])
def test_full_size_default_schedule_hash_equals_mpich(loop, gpu, case, path):
    name, P, n, digest, samples = next(c for c in CASES if c[0] == case)
    xs = fullsize_inputs(P, n)
    ins = [torch.from_numpy(x).to(gpu) for x in xs]
    del xs
    outs = [torch.full_like(t, float('nan')) for t in ins]
    with config(loop, tune=0, reference_order=1):
        if path == 'rccl_loopback':
            _loopback(loop, ins, outs, n)
        else:
            _thread_world_rccl(loop, ins, outs, n)
    torch.cuda.synchronize()
    _check(outs, digest, samples, (case, path))
    del ins, outs
    torch.cuda.empty_cache()


def test_full_size_c3_in_place_hash_equals_mpich(loop, gpu):
    """C3 in place (send == recv, as the keyed path runs a lone bucket) through the loopback."""
    name, P, n, digest, samples = next(c for c in CASES if c[1] == 8)
    bufs = [torch.from_numpy(x).to(gpu) for x in fullsize_inputs(P, n)]
    with config(loop, tune=0, reference_order=1):
        _loopback(loop, bufs, bufs, n)
    torch.cuda.synchronize()
    _check(bufs, digest, samples, (name, 'in_place'))
    del bufs
    torch.cuda.empty_cache()


def test_fullsize_inputs_are_the_generator_rule():
    """The regenerated inputs follow make_golden.py's rule (a cheap guard on the seed)."""
    a = fullsize_inputs(2, 8)
    want = np.random.default_rng(1234 + 7919).standard_normal(8).astype(np.float32)
    assert a[1].tobytes() == want.tobytes()
