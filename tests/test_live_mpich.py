"""Parity against MPICH run live (not only the committed golden vectors): random rank counts,
sizes on both sides of MPICH's 2048-byte algorithm switch and large messages, fp32 / fp64 /
int32. MPICH 3.3.2's MPI_Allreduce(MPI_SUM) runs through our driver
(oracle/mpi_allreduce_driver.c, one process per rank, as MPICommunicator.cc:14-28 calls it).

* CPU: the oracle's reference-order restatement (ddlo_fold_ref_order) equals MPICH bit for bit;
* GPU: the engine (P virtual ranks, reference_order 1, every schedule asked for) equals MPICH
  bit for bit.
Skipped where the image has no MPICH or the driver is not built (make -C oracle mpi)."""
import ctypes

import numpy as np
import pytest

from _helpers import DT_DOUBLE, DT_FLOAT, DT_INT32, config, live_mpich, live_mpich_available, random_input

needs_mpich = pytest.mark.skipif(not live_mpich_available(), reason='MPICH / oracle mpi driver not present')

# (P, dtype, n): 2048-byte switch at n = 512 fp32 / 256 fp64; large messages up to 4 MiB
CASES = [(3, DT_FLOAT, 700), (5, DT_FLOAT, 511), (5, DT_FLOAT, 512), (5, DT_FLOAT, 513), (5, DT_DOUBLE, 255),
         (5, DT_DOUBLE, 257), (6, DT_FLOAT, 3001), (7, DT_FLOAT, 100), (7, DT_DOUBLE, 9999), (5, DT_FLOAT, 1 << 20),
         (7, DT_FLOAT, 300_007), (8, DT_FLOAT, 65_537), (5, DT_INT32, 4099), (2, DT_FLOAT, 12_345),
         # beyond one node's GPUs, one host (fold trees of more than 16 inputs)
         (17, DT_FLOAT, 3000), (20, DT_FLOAT, 511), (33, DT_FLOAT, 4099), (33, DT_DOUBLE, 255)]


def _inputs(P, dt, n):
    return [random_input(dt, n, 4242 + 977 * r + n) for r in range(P)]


@needs_mpich
@pytest.mark.parametrize('P,dt,n', CASES)
def test_oracle_reference_order_vs_live_mpich(oracle, P, dt, n):
    xs = _inputs(P, dt, n)
    assert oracle.fold_ref_order(dt, xs).tobytes() == live_mpich(xs, dt).tobytes()


@pytest.mark.gpu
@needs_mpich
@pytest.mark.parametrize('algo', [0, 1, 2, 3])
def test_engine_reference_order_vs_live_mpich(lib, gpu, algo):
    import torch
    s = torch.cuda.current_stream().cuda_stream
    for P, dt, n in CASES:
        xs = _inputs(P, dt, n)
        want = live_mpich(xs, dt)
        ins = [torch.from_numpy(x).to(gpu) for x in xs]
        send = (ctypes.c_void_p * P)(*[t.data_ptr() for t in ins])
        with config(lib, algo=algo, reference_order=1, slice_bytes=256 << 10):
            assert lib.ddl_local_ring_allreduce(P, send, send, n, dt, 0, s) == 0, lib.ddl_last_error()
            torch.cuda.synchronize()
        for r, t in enumerate(ins):
            assert t.cpu().numpy().tobytes() == want.tobytes(), (P, dt, n, r)
