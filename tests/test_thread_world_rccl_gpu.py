"""The production executor, asynchronously, with its bytes handed to RCCL (VERDICT r3 missing #1 /
weak #2): the thread world of test_thread_world_gpu.py — P threads, each driving its own
RingExecutor::run_ (what ddl_allreduce runs at N > 1) — with ddl_testing_thread_transport(1), so
every matched send / receive pair moves through RcclTransport::group (the production transport
code) as a self send + self receive on a one-rank RCCL communicator, posted on the receiver's
stream after its wait on the sender's event. RCCL refuses two ranks of one host on one GPU, so within one process this is as close
to `RingExecutor` + `RcclTransport` at P > 1 as a one-GPU box allows: the same executor, the same
transport call, RCCL kernels carrying the data; only the peer (self) and who posts the pair differ.

Bar: as test_thread_world_gpu.py — MPICH golden vectors, oracle cases for every schedule, C3 / C4 /
C5 at full size, broadcast / allgatherv, race-free posted dependencies — and every test checks that
the pairs went through RCCL (the loopback pair counter moved)."""
import ctypes

import pytest

import test_batch_gpu as tb
import test_thread_world_gpu as tw
from _helpers import DT_DOUBLE, DT_FLOAT, DT_HALF, DT_INT32, NAME

pytestmark = pytest.mark.gpu


def _pairs(lib):
    v = ctypes.c_longlong(-1)
    assert lib.ddl_testing_thread_transport(1, ctypes.byref(v)) == 0, lib.ddl_last_error()
    return v.value


@pytest.fixture(scope='module')
def rccl_threads(lib, gpu):
    assert lib.ddl_rccl_loopback_init(0) == 0, lib.ddl_last_error()
    assert lib.ddl_testing_thread_transport(1, None) == 0, lib.ddl_last_error()
    yield lib
    assert lib.ddl_testing_thread_transport(0, None) == 0
    assert lib.ddl_rccl_loopback_finalize() == 0, lib.ddl_last_error()


@pytest.fixture
def through_rccl(rccl_threads):
    """Every test below must move bytes through RCCL."""
    before = _pairs(rccl_threads)
    yield
    assert _pairs(rccl_threads) > before, 'no send / receive pair went through RCCL'


@pytest.mark.parametrize('algo', [0, 1, 2, 3, 4])
def test_rccl_threads_mpich_golden(lib, gpu, through_rccl, algo):
    tw.test_thread_world_mpich_golden(lib, gpu, algo)


@pytest.mark.parametrize('P', [2, 3, 5, 8])
@pytest.mark.parametrize('algo,ref', [(0, 0), (1, 0), (2, 0), (3, 0), (1, 1), (2, 1), (3, 1), (4, 1)])
@pytest.mark.parametrize('dt', [DT_FLOAT, DT_DOUBLE, DT_INT32], ids=lambda d: NAME[d])
def test_rccl_threads_schedules_vs_oracle(lib, oracle, gpu, through_rccl, P, algo, ref, dt):
    tw.test_thread_world_schedules_vs_oracle(lib, oracle, gpu, P, algo, ref, dt)


@pytest.mark.parametrize('algo', [1, 4])
def test_rccl_threads_c3_full_size(lib, oracle, gpu, through_rccl, algo):
    tw.test_thread_world_c3_full_size(lib, oracle, gpu, algo)


def test_rccl_threads_c4_fp16_full_size(lib, oracle, gpu, through_rccl):
    tw.test_thread_world_c4_fp16_full_size(lib, oracle, gpu)


def test_rccl_threads_c5_full_4096_buckets_exact(lib, gpu, through_rccl):
    tw.test_thread_world_c5_full_4096_buckets_exact(lib, gpu)


@pytest.mark.parametrize('cap', [0, 1 << 20])
def test_rccl_threads_c5_sample_random_vs_oracle(lib, oracle, gpu, through_rccl, cap):
    tw.test_thread_world_c5_sample_random_vs_oracle(lib, oracle, gpu, cap)


@pytest.mark.parametrize('P', [2, 5, 8])
def test_rccl_threads_broadcast_allgatherv(lib, oracle, gpu, through_rccl, P):
    tw.test_thread_world_broadcast_allgatherv(lib, oracle, gpu, P)


def test_rccl_threads_repeated_calls(lib, oracle, gpu, through_rccl):
    tw.test_thread_world_repeated_calls_reuse_events(lib, oracle, gpu)


@pytest.mark.parametrize('P', [3, 8])
@pytest.mark.parametrize('algo,ref', [(0, 0), (1, 1), (4, 1)])
def test_rccl_threads_posted_dependencies_have_no_race(lib, gpu, through_rccl, P, algo, ref):
    tw.test_posted_dependencies_have_no_race(lib, gpu, P, algo, ref)


@pytest.mark.parametrize('P', [3, 8])
@pytest.mark.parametrize('dt', [DT_FLOAT, DT_HALF], ids=lambda d: NAME[d])
def test_rccl_threads_grouped_allreduce(lib, oracle, gpu, through_rccl, P, dt):
    """The grouped allreduce (RingExecutor::allreduce_batch: one group per tick for every bucket,
    batched folds) with its pairs through RCCL: every bucket bit for bit its own MPICH order."""
    tb.test_thread_batch_bit_exact_per_bucket(lib, oracle, gpu, P, 1, dt)
