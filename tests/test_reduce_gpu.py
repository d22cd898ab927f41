"""Per-hop reduce kernel (reduce_kernels.hip) vs the oracle's MPI_SUM operator: bit-exact for
every dtype (fp16/bf16: one rounding per add, identical to round(float(a)+float(b)))."""
import ctypes

import numpy as np
import pytest
import torch

from _helpers import ALL_DTYPES, DT_BFLOAT16, DT_FLOAT, DT_HALF, NAME, NP, random_input

pytestmark = pytest.mark.gpu

SIZES = [0, 1, 3, 4, 5, 63, 64, 65, 255, 256, 1000, 4097, 65_536 + 3, 1 << 20, (1 << 22) + 13]


def to_dev(x, dev):
    return torch.from_numpy(np.ascontiguousarray(x)).to(dev)


def from_dev(t, like):
    return t.cpu().numpy().view(like.dtype)


@pytest.mark.parametrize('dt', ALL_DTYPES, ids=lambda d: NAME[d])
@pytest.mark.parametrize('n', SIZES)
def test_sum2_bit_exact(lib, oracle, gpu, dt, n):
    a, b = random_input(dt, n, 11), random_input(dt, n, 12)
    ta, tb, to = to_dev(a, gpu), to_dev(b, gpu), torch.empty(max(n, 1), dtype=to_dev(a[:0], gpu).dtype, device=gpu)
    s = torch.cuda.current_stream().cuda_stream
    assert lib.ddl_reduce_sum2(to.data_ptr(), ta.data_ptr(), tb.data_ptr(), n, dt, s) == 0
    torch.cuda.synchronize()
    want = oracle.sum2(dt, a, b)
    assert from_dev(to[:n], a).tobytes() == want.tobytes()


@pytest.mark.parametrize('dt', ALL_DTYPES, ids=lambda d: NAME[d])
def test_reduce_local_in_place(lib, oracle, gpu, dt):
    n = 300_001
    a, b = random_input(dt, n, 21), random_input(dt, n, 22)
    ta, tb = to_dev(a, gpu), to_dev(b, gpu)
    assert lib.ddl_reduce_local(ta.data_ptr(), tb.data_ptr(), n, dt, torch.cuda.current_stream().cuda_stream) == 0
    torch.cuda.synchronize()
    assert from_dev(ta, a).tobytes() == oracle.sum2(dt, a, b).tobytes()


@pytest.mark.parametrize('variant', [-1, 0, 1, 2, 3, 4, 7, 8, 9, 15, 16, 19, 23, 24, 31])
@pytest.mark.parametrize('dt', [DT_FLOAT, DT_HALF, DT_BFLOAT16, 3, 2], ids=lambda d: str(d))
def test_variants_agree(lib, oracle, gpu, variant, dt):
    n = (1 << 20) + 77
    a, b = random_input(dt, n, 31), random_input(dt, n, 32)
    ta, tb = to_dev(a, gpu), to_dev(b, gpu)
    to = torch.empty_like(ta)
    assert lib.ddl_reduce_sum2_variant(variant, to.data_ptr(), ta.data_ptr(), tb.data_ptr(), n, dt,
                                       torch.cuda.current_stream().cuda_stream) == 0
    torch.cuda.synchronize()
    assert from_dev(to, a).tobytes() == oracle.sum2(dt, a, b).tobytes()


@pytest.mark.parametrize('variant', [32, 32 | 16, 32 | 19, 32 | 7, 96 | 7, 96 | 19])
@pytest.mark.parametrize('dt', [DT_FLOAT, DT_HALF, DT_BFLOAT16, 3, 2], ids=lambda d: str(d))
@pytest.mark.parametrize('n', [1, 7, 128 * 4 * 8 - 1, 128 * 4 * 8 + 5, (1 << 20) + 77])
def test_run_form_variants_agree(lib, oracle, gpu, variant, dt, n):
    """The run form of the two-input reduce (variant bit 32: a workgroup streams an 8-tile run of a,
    then of b; bit 64: 4-tile runs), in place and out of place, ragged lengths around a run."""
    a, b = random_input(dt, n, 33), random_input(dt, n, 34)
    ta, tb = to_dev(a, gpu), to_dev(b, gpu)
    to = torch.empty_like(ta)
    s = torch.cuda.current_stream().cuda_stream
    assert lib.ddl_reduce_sum2_variant(variant, to.data_ptr(), ta.data_ptr(), tb.data_ptr(), n, dt, s) == 0
    assert lib.ddl_reduce_sum2_variant(variant, ta.data_ptr(), ta.data_ptr(), tb.data_ptr(), n, dt, s) == 0
    torch.cuda.synchronize()
    want = oracle.sum2(dt, a, b).tobytes()
    assert from_dev(to, a).tobytes() == want and from_dev(ta, a).tobytes() == want


@pytest.mark.parametrize('offset', [1, 2, 3])
def test_misaligned_buffers(lib, oracle, gpu, offset):
    """Sub-tensor views that are not 16-byte aligned take the scalar path, same result."""
    n = 100_000
    a, b = random_input(DT_FLOAT, n + 8, 41), random_input(DT_FLOAT, n + 8, 42)
    ta, tb = to_dev(a, gpu), to_dev(b, gpu)
    to = torch.zeros_like(ta)
    av, bv, ov = ta[offset:offset + n], tb[offset:offset + n], to[offset:offset + n]
    assert lib.ddl_reduce_sum2(ov.data_ptr(), av.data_ptr(), bv.data_ptr(), n, DT_FLOAT,
                               torch.cuda.current_stream().cuda_stream) == 0
    torch.cuda.synchronize()
    want = oracle.sum2(DT_FLOAT, a[offset:offset + n], b[offset:offset + n])
    assert to.cpu().numpy()[offset:offset + n].tobytes() == want.tobytes()
    assert np.all(to.cpu().numpy()[:offset] == 0)


def test_special_values(lib, oracle, gpu):
    """inf, nan, signed zeros, denormals and fp16 overflow follow IEEE exactly as the oracle."""
    f = np.array([np.inf, -np.inf, np.nan, 0.0, -0.0, 1e-45, -1e-45, 3.4e38, 3.4e38, 1.0], np.float32)
    g = np.array([1.0, np.inf, 1.0, -0.0, -0.0, 1e-45, 1e-45, 3.4e38, -3.4e38, -1.0], np.float32)
    for dt, cast in ((DT_FLOAT, np.float32), (DT_HALF, np.float16)):
        a, b = f.astype(cast), g.astype(cast)
        if dt == DT_HALF:
            a = np.concatenate([a, np.array([65504, 6e-8, -6e-8], np.float16)])
            b = np.concatenate([b, np.array([16, 6e-8, 0], np.float16)])
        ta, tb = to_dev(a, gpu), to_dev(b, gpu)
        to = torch.empty_like(ta)
        assert lib.ddl_reduce_sum2(to.data_ptr(), ta.data_ptr(), tb.data_ptr(), a.size, dt,
                                   torch.cuda.current_stream().cuda_stream) == 0
        torch.cuda.synchronize()
        got, want = from_dev(to, a), oracle.sum2(dt, a, b)
        bits = np.uint16 if dt == DT_HALF else np.uint32
        nan = np.isnan(want)
        assert np.array_equal(np.isnan(got), nan)
        assert np.array_equal(got.view(bits)[~nan], want.view(bits)[~nan])


def test_int32_wraparound(lib, oracle, gpu):
    a = np.array([2 ** 31 - 1, -2 ** 31, -1, 123], np.int32)
    b = np.array([1, -1, 1, -123], np.int32)
    ta, tb = to_dev(a, gpu), to_dev(b, gpu)
    assert lib.ddl_reduce_local(ta.data_ptr(), tb.data_ptr(), 4, 3, torch.cuda.current_stream().cuda_stream) == 0
    torch.cuda.synchronize()
    assert ta.cpu().numpy().tolist() == [-2 ** 31, 2 ** 31 - 1, 0, 0]


def test_pack_unpack_roundtrip(lib, gpu):
    rng = np.random.default_rng(5)
    sizes = [int(s) for s in rng.integers(1, 70_000, size=150)] + [4, 16, 256, 4096]
    srcs = [torch.from_numpy(rng.integers(0, 255, size=s, dtype=np.uint8)).to(gpu) for s in sizes]
    total = sum((s + 255) // 256 * 256 for s in sizes)
    fused = torch.zeros(total, dtype=torch.uint8, device=gpu)
    P = ctypes.c_void_p * len(sizes)
    S = ctypes.c_size_t * len(sizes)
    stream = torch.cuda.current_stream().cuda_stream
    assert lib.ddl_pack(fused.data_ptr(), P(*[t.data_ptr() for t in srcs]), S(*sizes), len(sizes), stream) == 0
    outs = [torch.zeros_like(t) for t in srcs]
    assert lib.ddl_unpack(P(*[t.data_ptr() for t in outs]), fused.data_ptr(), S(*sizes), len(sizes), stream) == 0
    torch.cuda.synchronize()
    off = 0
    f = fused.cpu().numpy()
    for s, src, out in zip(sizes, srcs, outs):
        assert np.array_equal(f[off:off + s], src.cpu().numpy())
        assert torch.equal(out, src)
        off += (s + 255) // 256 * 256


@pytest.mark.parametrize('case', ['dense_tiny', 'many_segments', 'unaligned', 'zero_lengths', 'empty_runs'])
def test_pack_unpack_layouts(lib, gpu, case):
    """Segment tables the tile index must resolve: one-tile segments (128 segments per index
    block), > 4096 segments, byte-misaligned pointers (byte path), zero-length segments sharing a
    tile with their successor, and runs of 300 empty segments inside one 128-tile block (more
    than a byte's reach: the int32 index fallback)."""
    rng = np.random.default_rng(sum(map(ord, case)))
    if case == 'dense_tiny':
        sizes = [int(s) for s in rng.integers(1, 300, size=3000)]
    elif case == 'many_segments':
        sizes = [int(s) for s in rng.integers(1, 5000, size=9000)]
    elif case == 'unaligned':
        sizes = [int(s) for s in rng.integers(1, 40_000, size=200)]
    elif case == 'empty_runs':
        sizes = ([3000, 17] + [0] * 300 + [5, 2048]) * 3 + [70_001]
    else:
        sizes = [0, 5, 0, 0, 300, 0, 70_000, 0, 17]
    pool = torch.from_numpy(rng.integers(0, 255, size=sum(sizes) + 16 * len(sizes) + 64, dtype=np.uint8)).to(gpu)
    outpool = torch.zeros_like(pool)
    offs, o = [], 3 if case == 'unaligned' else 0
    for s in sizes:
        offs.append(o)
        o += s + (int(rng.integers(1, 16)) if case == 'unaligned' else 0)
    total = sum((s + 255) // 256 * 256 for s in sizes)
    fused = torch.zeros(max(total, 1), dtype=torch.uint8, device=gpu)
    P = ctypes.c_void_p * len(sizes)
    S = ctypes.c_size_t * len(sizes)
    stream = torch.cuda.current_stream().cuda_stream
    assert lib.ddl_pack(fused.data_ptr(), P(*[pool.data_ptr() + x for x in offs]), S(*sizes), len(sizes), stream) == 0
    assert lib.ddl_unpack(P(*[outpool.data_ptr() + x for x in offs]), fused.data_ptr(), S(*sizes), len(sizes),
                          stream) == 0
    torch.cuda.synchronize()
    f, src, dst = fused.cpu().numpy(), pool.cpu().numpy(), outpool.cpu().numpy()
    off = 0
    covered = np.zeros(dst.size, dtype=bool)
    for s, x in zip(sizes, offs):
        assert np.array_equal(f[off:off + s], src[x:x + s])
        assert np.array_equal(dst[x:x + s], src[x:x + s])
        covered[x:x + s] = True
        off += (s + 255) // 256 * 256
    assert not dst[~covered].any()  # unpack writes nothing between or past the segments


@pytest.mark.parametrize('dt', [1, 2, 3, 9, 14, 19, 23])
@pytest.mark.parametrize('nb', [1, 2, 7, 15])
@pytest.mark.parametrize('n,misalign', [(1, 0), (4099, 0), (300_001, 0), (10_007, 1)])
def test_reduce_fold_kernel(lib, oracle, gpu, dt, nb, n, misalign):
    """k_sumN_tile / k_sumN_scalar alone: out = a + x_0 + ... + x_{nb-1} vs the oracle's fold
    (fp16/bf16: fp32 accumulation, one rounding), vector and misaligned paths, ragged tails."""
    from _helpers import random_input
    xs = [random_input(dt, n + misalign, 900 + 13 * i + dt) for i in range(nb + 1)]
    ts = [to_dev(x, gpu) for x in xs]
    es = xs[0].itemsize
    ptrs = [t.data_ptr() + misalign * es for t in ts]
    out = torch.zeros_like(ts[0])
    P = ctypes.c_void_p * nb
    st = lib.ddl_reduce_fold(out.data_ptr() + misalign * es, ptrs[0], P(*ptrs[1:]), nb, n, dt,
                             torch.cuda.current_stream().cuda_stream)
    assert st == 0, lib.ddl_last_error()
    torch.cuda.synchronize()
    want = oracle.fold(dt, [x[misalign:] for x in xs])
    got = out.cpu().numpy().view(xs[0].dtype)[misalign:]
    assert got.tobytes() == want.tobytes()


@pytest.mark.parametrize('dt', [1, 2, 3, 14])
@pytest.mark.parametrize('nb', [1, 2, 3, 4, 5, 6, 7, 9, 12, 15])
@pytest.mark.parametrize('order', [1, 2])
@pytest.mark.parametrize('n,misalign', [(1, 0), (300_001, 0), (10_007, 1)])
def test_reduce_fold_ordered_kernel(lib, oracle, gpu, dt, nb, order, n, misalign):
    """The reference-order folds alone (ddl_reduce_fold_ordered): MPICH's pre-fold + pairwise
    tree (order 1) and binomial tree (order 2) over nb + 1 inputs vs the oracle's restatement,
    vector and misaligned paths; fp16/bf16 keep the fp32 left fold."""
    from _helpers import random_input
    xs = [random_input(dt, n + misalign, 700 + 17 * i + dt) for i in range(nb + 1)]
    ts = [to_dev(x, gpu) for x in xs]
    es = xs[0].itemsize
    ptrs = [t.data_ptr() + misalign * es for t in ts]
    out = torch.zeros_like(ts[0])
    P = ctypes.c_void_p * nb
    st = lib.ddl_reduce_fold_ordered(out.data_ptr() + misalign * es, ptrs[0], P(*ptrs[1:]), nb, n, dt, order,
                                     torch.cuda.current_stream().cuda_stream)
    assert st == 0, lib.ddl_last_error()
    torch.cuda.synchronize()
    want = oracle.fold_ref_order(dt, [x[misalign:] for x in xs], 4096 if order == 1 else 0)
    got = out.cpu().numpy().view(xs[0].dtype)[misalign:]
    assert got.tobytes() == want.tobytes()


# the run form of the fold (reduce_kernels.hip k_sumN_run: chunks from 4 MiB with 7+ inputs, a workgroup walks
# the inputs one at a time over a 16 KiB run): every dtype, 2..16 inputs, the left fold and MPICH's
# tree, chunk sizes a whole number of runs plus a ragged tail and not
RUN_BYTES = [(9 << 20) + 16 * 1024 * 3, (9 << 20) + 4096 + 48]


@pytest.mark.parametrize('dt', [1, 2, 3, 9, 14, 19, 23])
@pytest.mark.parametrize('nb', [1, 2, 4, 7, 9, 15])
@pytest.mark.parametrize('order', [0, 1])
@pytest.mark.parametrize('nbytes', RUN_BYTES + [4100 * 4, 1 << 20], ids=['whole_runs+tail', 'ragged', 'small',
                                                                         '1MiB'])
def test_reduce_fold_run_form(lib, oracle, gpu, dt, nb, order, nbytes):
    """The run form (the default from 4 MiB at 7+ inputs) forced for every width and size (config
    fold_form 2), so its tails are checked at sizes of one run and less too."""
    from _helpers import config
    es = {1: 4, 2: 8, 3: 4, 9: 8, 14: 2, 19: 2, 23: 8}[dt]
    n = nbytes // es + (es < 8) * 3  # + a tail shorter than one 16-byte vector (for es < 8)
    with config(lib, fold_form=2):
        _fold_check(lib, oracle, gpu, dt, nb, order, n, es)


@pytest.mark.parametrize('dt', [1, 14])
@pytest.mark.parametrize('nb', [2, 7])
def test_reduce_fold_tile_form_forced_large(lib, oracle, gpu, dt, nb):
    """config fold_form 1 keeps the tile form at large chunks (the A/B the bench reports)."""
    from _helpers import config
    es = 4 if dt == 1 else 2
    with config(lib, fold_form=1):
        _fold_check(lib, oracle, gpu, dt, nb, 1, RUN_BYTES[1] // es + 3, es)


def _fold_check(lib, oracle, gpu, dt, nb, order, n, es):
    xs = [random_input(dt, n, 1300 + 7 * i + dt) for i in range(nb + 1)]
    ts = [to_dev(x, gpu) for x in xs]
    out = torch.zeros_like(ts[0])
    P = ctypes.c_void_p * nb
    s = torch.cuda.current_stream().cuda_stream
    ptrs = [t.data_ptr() for t in ts]
    if order == 0:
        st = lib.ddl_reduce_fold(out.data_ptr(), ptrs[0], P(*ptrs[1:]), nb, n, dt, s)
    else:
        st = lib.ddl_reduce_fold_ordered(out.data_ptr(), ptrs[0], P(*ptrs[1:]), nb, n, dt, 1, s)
    assert st == 0, lib.ddl_last_error()
    torch.cuda.synchronize()
    want = oracle.fold(dt, xs) if order == 0 else oracle.fold_ref_order(dt, xs, 4096)
    got = out.cpu().numpy().view(xs[0].dtype)
    assert got.tobytes() == want.tobytes(), np.flatnonzero(got.view(np.uint8) != want.view(np.uint8))[:8]


def test_reduce_fold_ordered_rejects_bad_order(lib, gpu):
    x = torch.zeros(16, device=gpu)
    P = ctypes.c_void_p * 1
    assert lib.ddl_reduce_fold_ordered(x.data_ptr(), x.data_ptr(), P(x.data_ptr()), 1, 16, 1, 3,
                                       torch.cuda.current_stream().cuda_stream) == 3


# C2's headline sizes: the bench's 256 MiB and 1 GiB launches, at full
# size, and a size in every band default_variant picks (reduce_kernels.hip kReduceBands: below 12 MiB
# the tile form with plain loads; 12-22 MiB the run form, non-temporal loads; 22-42 MiB the run form,
# plain loads; 42-96 MiB the run form, non-temporal loads; 96-256 MiB the tile form, non-temporal
# loads — all with write-through stores; from 256 MiB all non-temporal). Integer-valued fp32 in
# (-2^22, 2^22): every sum is exact in fp32, so the WHOLE output is checked against the exact sum;
# then random data against the oracle's MPI_SUM on a strided sample of the same launch.
C2_SIZES = [(8 << 20) // 4 + 9, (16 << 20) // 4 + 7, (32 << 20) // 4 + 3, (64 << 20) // 4 + 5,
            (100 << 20) // 4 + 1, (256 << 20) // 4, (1 << 30) // 4 + 13]


@pytest.mark.parametrize('in_place', [True, False], ids=['local', 'sum2'])
@pytest.mark.parametrize('n', C2_SIZES, ids=lambda n: f'{n * 4 >> 20}MiB+{n % 1024}')
def test_c2_headline_sizes_exact(lib, oracle, gpu, n, in_place):
    s = torch.cuda.current_stream().cuda_stream
    g = torch.Generator(device=gpu).manual_seed(n)
    a = torch.randint(-(1 << 22), 1 << 22, (n,), device=gpu, generator=g, dtype=torch.int32).float()
    b = torch.randint(-(1 << 22), 1 << 22, (n,), device=gpu, generator=g, dtype=torch.int32).float()
    want = a + b  # exact: |a + b| < 2^23
    if in_place:
        assert lib.ddl_reduce_local(a.data_ptr(), b.data_ptr(), n, DT_FLOAT, s) == 0, lib.ddl_last_error()
        out = a
    else:
        out = torch.full_like(a, float('nan'))
        assert lib.ddl_reduce_sum2(out.data_ptr(), a.data_ptr(), b.data_ptr(), n, DT_FLOAT, s) == 0
    torch.cuda.synchronize()
    bad = torch.nonzero(out.view(torch.int32) != want.view(torch.int32))
    assert bad.numel() == 0, f'{bad.numel()} elements differ, first at {bad[:4].flatten().tolist()}'
    del a, b, out, want
    # random data: the oracle on a strided sample plus the tail
    x = torch.randn(n, device=gpu, generator=g)
    y = torch.randn(n, device=gpu, generator=g)
    z = torch.empty_like(x)
    assert lib.ddl_reduce_sum2(z.data_ptr(), x.data_ptr(), y.data_ptr(), n, DT_FLOAT, s) == 0
    torch.cuda.synchronize()
    idx = torch.cat([torch.arange(0, n, 4099, device=gpu), torch.arange(max(0, n - 4096), n, device=gpu)])
    xs, ys, zs = (t[idx].cpu().numpy() for t in (x, y, z))
    assert zs.tobytes() == oracle.sum2(DT_FLOAT, xs, ys).tobytes()
    del x, y, z
    torch.cuda.empty_cache()
