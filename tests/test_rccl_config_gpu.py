"""RCCL communicator configuration: config rccl_min_ctas / rccl_max_ctas reach
ncclCommInitRankConfig / ncclCommSplit as ncclConfig_t.minCTAs / maxCTAs. A one-rank loopback
communicator created under each setting (and a split of it) carries C3 at full size — 8 virtual
ranks x 64 Mi fp32, the default schedule through the engine's RcclTransport — to MPICH 3.3.2's
own output (tests/golden/golden_fullsize.json), bit for bit on every rank."""
import ctypes

import pytest
import torch

from _helpers import DT_FLOAT, config, fullsize_cases, fullsize_inputs, sha256

pytestmark = pytest.mark.gpu

SETTINGS = [(0, 0), (1, 1), (4, 8), (16, 32), (64, 64)]


@pytest.mark.parametrize('lo,hi', SETTINGS, ids=lambda v: str(v))
def test_loopback_communicator_per_cta_setting_runs_c3_bit_exact(lib, gpu, lo, hi):
    name, P, n, digest, _ = next(c for c in fullsize_cases() if c[1] == 8)
    ins = [torch.from_numpy(x).to(gpu) for x in fullsize_inputs(P, n)]
    outs = [torch.full_like(t, float('nan')) for t in ins]
    send = (ctypes.c_void_p * P)(*[t.data_ptr() for t in ins])
    recv = (ctypes.c_void_p * P)(*[t.data_ptr() for t in outs])
    s = torch.cuda.current_stream().cuda_stream
    with config(lib, rccl_min_ctas=lo, rccl_max_ctas=hi, tune=0, reference_order=1):
        assert lib.ddl_rccl_loopback_init(0) == 0, lib.ddl_last_error()
        try:
            assert lib.ddl_rccl_loopback_allreduce(P, send, recv, n, DT_FLOAT, s) == 0, lib.ddl_last_error()
            torch.cuda.synchronize()
            for r, o in enumerate(outs):
                assert sha256(o.cpu().numpy()) == digest, ('init', lo, hi, r)
            outs[0].fill_(float('nan'))
            rk, sz = ctypes.c_int(-1), ctypes.c_int(-1)
            assert lib.ddl_rccl_loopback_split(0, 0, ctypes.byref(rk), ctypes.byref(sz)) == 0, lib.ddl_last_error()
            assert (rk.value, sz.value) == (0, 1)
            assert lib.ddl_rccl_loopback_allreduce(P, send, recv, n, DT_FLOAT, s) == 0, lib.ddl_last_error()
            torch.cuda.synchronize()
            for r, o in enumerate(outs):
                assert sha256(o.cpu().numpy()) == digest, ('split', lo, hi, r)
        finally:
            assert lib.ddl_rccl_loopback_finalize() == 0, lib.ddl_last_error()
    del ins, outs
    torch.cuda.empty_cache()


def test_min_above_max_is_refused_at_creation(lib, gpu):
    with config(lib, rccl_min_ctas=8, rccl_max_ctas=4):
        assert lib.ddl_rccl_loopback_init(0) == 3
        assert b'rccl_min_ctas' in lib.ddl_last_error()
