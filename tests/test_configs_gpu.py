"""BASELINE.json's multi-GPU configs at their full shapes, on one GPU with 8 virtual ranks whose
point-to-point moves go through real RCCL (ddl_rccl_loopback_*, the engine's RcclTransport):

  C3  fp32, one 256 MiB bucket per rank  — random data, the default (reference-order) schedule,
      every rank bit-exact vs the MPICH-order oracle (ddlo_fold_ref_order);
  C4  fp16, 1 GiB per rank as 64 x 16 MiB buckets — within the direct schedule's single-rounding
      bound |y - sum| <= ulp16(y)/2 + (P-1) * 2^-24 * sum|x|, and bit-exact vs the oracle's fp16
      rule on every bucket (the reference rejects fp16: MPICH has no fp16 sum to pin it);
  C5  4096 mixed fp32/fp16 buckets of 4 KiB - 4 MiB (2.4 GB per rank) through the keyed data
      plane's pieces — per dtype group in key order: one-launch pack into the fusion buffer,
      allreduce, one-launch unpack — exact on integer-valued data at full size, and bit-exact vs
      the oracle on random data for a 512-bucket sample.
"""
import ctypes

import numpy as np
import pytest
import torch

from _helpers import DT_FLOAT, DT_HALF, config, fp16_single_rounding_bound, random_input

pytestmark = pytest.mark.gpu
P = 8


@pytest.fixture(scope='module')
def loop(lib, gpu):
    st = lib.ddl_rccl_loopback_init(0)
    assert st == 0, lib.ddl_last_error()
    yield lib
    assert lib.ddl_rccl_loopback_finalize() == 0, lib.ddl_last_error()


def _allreduce(lib, ins, outs, n, dt):
    send = (ctypes.c_void_p * P)(*[t.data_ptr() for t in ins])
    recv = (ctypes.c_void_p * P)(*[t.data_ptr() for t in outs])
    st = lib.ddl_rccl_loopback_allreduce(P, send, recv, n, dt, torch.cuda.current_stream().cuda_stream)
    assert st == 0, lib.ddl_last_error()


def test_c3_reference_order_full_size(loop, oracle, gpu):
    """C3: 8 x 256 MiB random fp32, tuner off, default schedule and order, out of place."""
    n = 64 << 20
    xs = [random_input(DT_FLOAT, n, 777 + r) for r in range(P)]
    want = oracle.fold_ref_order(DT_FLOAT, xs).tobytes()
    ins = [torch.from_numpy(x).to(gpu) for x in xs]
    outs = [torch.empty_like(t) for t in ins]
    with config(loop, tune=0):
        _allreduce(loop, ins, outs, n, DT_FLOAT)
    torch.cuda.synchronize()
    for r, o in enumerate(outs):
        assert o.cpu().numpy().tobytes() == want, r


def test_c4_fp16_64x16mib_tolerance(loop, oracle, gpu):
    """C4: 64 buckets of 16 MiB fp16 per rank (1 GiB), N(0,1)*0.1, in place, default
    schedule (direct at P = 8: all 8 inputs folded in fp32, one rounding). Every rank within the
    single-rounding bound ulp16(y)/2 + (P-1)*2^-24*sum|x| of the exact (fp64) sum, all ranks
    identical, and every bucket bit-exact vs the oracle's fp16 rule (MPICH order in fp32, one
    rounding) — a regression to per-hop rounding fails both."""
    nb = (16 << 20) // 2
    g = torch.Generator(device=gpu).manual_seed(4)
    worst = 0.0
    with config(loop, tune=0):
        for b in range(64):
            ins = [(torch.randn(nb, device=gpu, generator=g) * 0.1).half() for _ in range(P)]
            want = oracle.fold_ref_order(DT_HALF, [t.cpu().numpy() for t in ins])
            x64 = torch.stack(ins).double()
            exact, mag = x64.sum(0), x64.abs().sum(0)
            del x64
            _allreduce(loop, ins, ins, nb, DT_HALF)
            bound = fp16_single_rounding_bound(P, ins[0], mag)
            err = (ins[0].double() - exact).abs()
            assert bool((err <= bound).all()), b
            worst = max(worst, float((err / bound.clamp_min(1e-30)).max()))
            assert ins[0].cpu().numpy().tobytes() == want.tobytes(), b
            for t in ins[1:]:
                assert torch.equal(t, ins[0])
    assert worst <= 1.0


def _c5_buckets(k, seed=5, max_bytes=4 << 20):
    rng = np.random.default_rng(seed)
    sizes = (np.exp(rng.uniform(np.log(4096), np.log(max_bytes), size=k)).astype(np.int64) // 256) * 256
    half = rng.random(k) < 0.5
    return [(int(sizes[i]) // (2 if half[i] else 4), DT_HALF if half[i] else DT_FLOAT) for i in range(k)]


def _keyed_data_plane(lib, per_rank, buckets, gpu):
    """The keyed path's data plane for P ranks, per dtype group (ascending enum, keys
    grad_%05d in order): ddl_pack -> RCCL-loopback allreduce of the fusion buffers -> ddl_unpack."""
    outs = [[torch.empty_like(t) for t in ts] for ts in per_rank]
    s = torch.cuda.current_stream().cuda_stream
    for dt in sorted({d for _, d in buckets}):
        idx = [i for i, (_, d) in enumerate(buckets) if d == dt]  # key order = index order
        es = 2 if dt == DT_HALF else 4
        nbytes = [buckets[i][0] * es for i in idx]
        flat = sum((b + 255) // 256 * 256 for b in nbytes)
        m = len(idx)
        Sz, Vp = ctypes.c_size_t * m, ctypes.c_void_p * m
        fused = [torch.empty(flat, dtype=torch.uint8, device=gpu) for _ in range(P)]
        for r in range(P):
            assert lib.ddl_pack(fused[r].data_ptr(), Vp(*[per_rank[r][i].data_ptr() for i in idx]), Sz(*nbytes), m,
                                s) == 0, lib.ddl_last_error()
        _allreduce(lib, fused, fused, flat // es, dt)
        for r in range(P):
            assert lib.ddl_unpack(Vp(*[outs[r][i].data_ptr() for i in idx]), fused[r].data_ptr(), Sz(*nbytes), m,
                                  s) == 0, lib.ddl_last_error()
        del fused
    torch.cuda.synchronize()
    return outs


def test_c5_full_4096_buckets_exact(loop, gpu):
    """C5 at full size (4096 buckets, ~2.4 GB per rank, 8 ranks): integer-valued data (|x| <= 8,
    sums exact in fp16 and fp32), so every rank must equal the exact sum bit for bit."""
    buckets = _c5_buckets(4096)
    g = torch.Generator(device=gpu).manual_seed(55)
    tdt = {DT_FLOAT: torch.float32, DT_HALF: torch.float16}
    per_rank = [[torch.randint(-8, 9, (n,), device=gpu, generator=g).to(tdt[dt]) for n, dt in buckets]
                for _ in range(P)]
    with config(loop, tune=0):
        outs = _keyed_data_plane(loop, per_rank, buckets, gpu)
    for i in range(len(buckets)):
        want = torch.stack([per_rank[r][i] for r in range(P)]).float().sum(0).to(per_rank[0][i].dtype)
        for r in range(P):
            assert torch.equal(outs[r][i], want), (i, r)


def test_c5_sample_random_vs_oracle(loop, oracle, gpu):
    """512 buckets of the C5 distribution (capped at 256 KiB) with random data: every rank equals
    the oracle's MPICH order for the group's message, fp16 folded in fp32 in rank order."""
    buckets = _c5_buckets(512, seed=6, max_bytes=256 << 10)
    xs = [[random_input(dt, n, 10_000 * r + i) for i, (n, dt) in enumerate(buckets)] for r in range(P)]
    per_rank = [[torch.from_numpy(x.view(np.int16) if x.dtype == np.float16 else x).to(gpu) for x in row]
                for row in xs]
    per_rank = [[t.view(torch.float16) if t.dtype == torch.int16 else t for t in row] for row in per_rank]
    with config(loop, tune=0):
        outs = _keyed_data_plane(loop, per_rank, buckets, gpu)
    for i, (n, dt) in enumerate(buckets):
        want = oracle.fold_ref_order(dt, [xs[r][i] for r in range(P)], 1 << 30).tobytes()
        for r in range(P):
            assert outs[r][i].cpu().numpy().tobytes() == want, (i, r)
