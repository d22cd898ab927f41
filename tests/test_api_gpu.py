"""The reference's operator surface on the GPU at world size 1 (one process per GPU):
Communicator, allreduce / allreduce_gradient, keyed async requests with fusion, the
data-parallel optimizer wrapper. At size 1 the sum is the tensor itself (the reference hangs
there; the build defines out = in)."""
import ctypes
import gc
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope='module')
def world(gpu):
    from ddl.torch.communicator import Communicator
    return Communicator.world()


def test_world_communicator(world, lib):
    assert world.rank == 0 and world.size == 1
    assert world.id == lib.world_communicator() != 0


def test_allreduce_returns_new_tensor(world):
    from ddl.torch.tensor_communicate import allreduce
    x = torch.randn(1000, 7, device='cuda')
    y = allreduce(x, world)
    assert y.data_ptr() != x.data_ptr() and torch.equal(x, y)


def test_allreduce_host_tensor(world):
    from ddl.torch.tensor_communicate import allreduce
    x = torch.randn(4099)
    y = allreduce(x, world)
    assert not y.is_cuda and torch.equal(x, y)


@pytest.mark.parametrize('chunk', [4096, 1 << 20, 32 << 20])
@pytest.mark.parametrize('n,dtype', [(1, torch.float32), (1000, torch.float16), (3_000_001, torch.float32),
                                     (777_777, torch.int64)])
def test_allreduce_host_pipeline(world, lib, chunk, n, dtype):
    """Chunked H2D -> ring -> D2H pipeline (pageable input registered for the call), whole chunks."""
    from ddl.torch.cpp_backend import check
    from ddl.torch.util import ddl_dtype
    old = lib.ddl_get_config(b'host_chunk_bytes')
    assert lib.ddl_set_config(b'host_chunk_bytes', chunk) == 0
    try:
        x = (torch.randn(n) * 1000).to(dtype)
        y = torch.zeros_like(x)
        check(lib.ddl_allreduce_host(world.id, x.data_ptr(), y.data_ptr(), n, ddl_dtype(x), 0), 'host')
        assert torch.equal(x, y)
        z = x.clone()  # in place
        check(lib.ddl_allreduce_host(world.id, z.data_ptr(), z.data_ptr(), n, ddl_dtype(z), 0), 'host')
        assert torch.equal(x, z)
    finally:
        lib.ddl_set_config(b'host_chunk_bytes', old)


def test_allreduce_gradient_mean(world):
    from ddl.torch.tensor_communicate import allreduce_gradient
    x = torch.randn(333, device='cuda', dtype=torch.float16)
    assert torch.equal(allreduce_gradient(x, world), x)


def test_unsupported_dtype_raises(world):
    from ddl.torch.tensor_communicate import allreduce
    with pytest.raises(TypeError):
        allreduce(torch.ones(4, dtype=torch.int8, device='cuda'), world)


@pytest.mark.parametrize('threshold', [(1 << 31) - 1, 4096 + 1, 777])
def test_keyed_requests_fused(world, lib, threshold):
    """Many keyed requests of mixed dtypes: negotiated (size 1: all pending), grouped by dtype,
    fused into plans capped at the threshold, packed/unpacked — outputs equal inputs."""
    from ddl.torch.tensor_communicate import allreduce_async, wait_all
    old = lib.ddl_get_config(b'fusion_threshold_bytes')
    assert lib.ddl_set_config(b'fusion_threshold_bytes', threshold) == 0
    try:
        rng = np.random.default_rng(0)
        tensors, handles = [], []
        for i in rng.permutation(200):
            n = int(rng.integers(0, 5000))
            dt = [torch.float32, torch.float16, torch.int32, torch.bfloat16, torch.float64][i % 5]
            t = (torch.randn(n, device='cuda') * 100).to(dt)
            tensors.append(t)
            handles.append(allreduce_async(t, f'grad_{i:05d}', world))
        for t, h in zip(tensors, handles):
            assert torch.equal(h.wait(timeout=60), t)
        wait_all(world)
    finally:
        lib.ddl_set_config(b'fusion_threshold_bytes', old)


def test_keyed_batch_c5_shape(world, lib):
    """C5 shape: the full 4096 buckets, byte sizes log-uniform in [4 KiB, 4 MiB]
    rounded to 256 B, fp32/fp16 mixed, keys grad_%05d in random order — one batch, with the
    one-rank shortcut OFF, so negotiation, dtype groups, plans, the fusion pipeline's pack ->
    allreduce -> unpack all run. The oracle at one rank is the input itself (MPI_Allreduce of
    one rank); the 8-rank data plane of the same set is tests/test_configs_gpu.py."""
    from ddl.torch.tensor_communicate import allreduce_async_batch
    rng = np.random.default_rng(42)
    k = 4096
    sizes = np.exp(rng.uniform(np.log(4096), np.log(4 << 20), size=k)).astype(np.int64) // 256 * 256
    tensors, names = [], []
    for i in rng.permutation(k):
        dt = torch.float32 if rng.random() < 0.5 else torch.float16
        n = int(sizes[i]) // (4 if dt == torch.float32 else 2)
        tensors.append(torch.randn(n, device='cuda').to(dt))
        names.append(f'grad_{i:05d}')
    old = lib.ddl_get_config(b'one_rank_shortcut')
    try:
        assert lib.ddl_set_config(b'one_rank_shortcut', 0) == 0
        hs = allreduce_async_batch(tensors, names, world)
        for t, h in zip(tensors, hs):
            assert torch.equal(h.wait(60), t)
    finally:
        lib.ddl_set_config(b'one_rank_shortcut', old)


def test_keyed_batch_duplicate_rejected_atomically(world):
    from ddl.torch.cpp_backend import DDLError
    from ddl.torch.tensor_communicate import allreduce_async_batch
    ts = [torch.randn(8, device='cuda') for _ in range(3)]
    with pytest.raises(DDLError) as e:
        allreduce_async_batch(ts, ['x1', 'x2', 'x1'], world)
    assert e.value.status == 7
    hs = allreduce_async_batch(ts, ['x1', 'x2', 'x3'], world)  # nothing of the failed batch stuck
    for t, h in zip(ts, hs):
        assert torch.equal(h.wait(60), t)


def test_keyed_duplicate_key_rejected(world):
    from ddl.torch.cpp_backend import DDLError
    from ddl.torch.tensor_communicate import allreduce_async
    # hold the handler busy is not needed: a duplicate pending key is rejected at submit when
    # the first one is still registered; submit twice quickly and accept either outcome of the
    # race, but a reject must carry DUPLICATE_KEY.
    t = torch.randn(10, device='cuda')
    h = allreduce_async(t, 'dup_key', world)
    try:
        h2 = allreduce_async(t, 'dup_key', world)
        h2.wait(60)
    except DDLError as e:
        assert e.status == 7
    h.wait(60)


def test_done_callbacks_fire_in_reference_order(world, lib):
    """done() order: dtype groups ascending (float32=1 < float64=2 < int32=3 < half=19),
    keys lexicographic inside a group (MPIRingTokenCommunication.cc:105-157, 735-749)."""
    from ddl.torch import cpp_backend as cb
    order = []

    @cb.DONE_FN
    def done(status, user):
        order.append(user)

    api = cb.CPPBackend.c_api()
    keep = []
    block = torch.cuda.Stream()
    # a fusion window so every request registers before the handler proposes the round
    assert api.ddl_set_config(b'cycle_time_us', 300_000) == 0
    with torch.cuda.stream(block):
        specs = [('b', torch.float16), ('a', torch.float64), ('c', torch.float32), ('a', torch.float32),
                 ('z', torch.int32), ('m', torch.float16)]
        for i, (k, dt) in enumerate(specs):
            t = torch.ones(100, device='cuda', dtype=dt)
            keep.append(t)
            from ddl.torch.util import ddl_dtype
            st = api.ddl_allreduce_submit(world.id, f'{k}{i}'.encode(), t.data_ptr(), t.data_ptr(), t.numel(),
                                          ddl_dtype(t), 0, block.cuda_stream, done, i + 1)
            assert st == 0
    assert api.ddl_wait_all(world.id) == 0
    api.ddl_set_config(b'cycle_time_us', 0)
    order = [u - 1 for u in order]
    names = [f"{specs[i][0]}{i}" for i in order]
    dts = [specs[i][1] for i in order]
    rank = {torch.float32: 1, torch.float64: 2, torch.int32: 3, torch.float16: 19}
    assert [rank[d] for d in dts] == sorted(rank[d] for d in dts)
    for d in set(dts):
        grp = [n for n, x in zip(names, dts) if x == d]
        assert grp == sorted(grp)
    assert len(order) == len(specs)


@pytest.mark.parametrize('pipelined', [1, 0])
def test_keyed_rounds_pipelined(world, lib, data_plane_at_one_rank, pipelined):
    """Rounds back to back with the data plane on: with pipeline_rounds = 1 the completion
    thread fires round n's done() calls while the engine thread takes and enqueues round n+1
    (its pack / allreduce / unpack queued behind round n's on the same streams). Every output
    equals its input, every done() fires once with status 0, and done() order across rounds is
    the submission order (batches keyed so their keys sort in submission order, one dtype)."""
    from ddl.torch import cpp_backend as cb
    from ddl.torch.util import ddl_dtype
    assert lib.ddl_set_config(b'pipeline_rounds', pipelined) == 0
    order, statuses = [], []

    @cb.DONE_FN
    def done(status, user):
        order.append(user)
        statuses.append(status)

    api = cb.CPPBackend.c_api()
    stream = torch.cuda.current_stream()
    rng = np.random.default_rng(11 + pipelined)
    keep, want, uid = [], {}, 0
    try:
        for b in range(24):
            k = int(rng.integers(1, 40))
            ts = [torch.randn(int(rng.integers(1, 200_000)), device='cuda') for _ in range(k)]
            outs = [t if j % 2 else torch.zeros_like(t) for j, t in enumerate(ts)]
            keys = [f'round{b:03d}_{j:03d}'.encode() for j in range(k)]
            V = ctypes.c_void_p * k
            st = api.ddl_allreduce_submit_batch(
                world.id, k, (ctypes.c_char_p * k)(*keys), V(*[t.data_ptr() for t in ts]),
                V(*[o.data_ptr() for o in outs]), (ctypes.c_size_t * k)(*[t.numel() for t in ts]),
                (ctypes.c_int * k)(*[ddl_dtype(t) for t in ts]), 0, stream.cuda_stream, done, None)
            assert st == 0
            # the batch's user pointers are None: identify by key order instead (one done per key)
            for j in range(k):
                want[uid] = (ts[j].clone(), outs[j])
                uid += 1
            keep.append((ts, outs))
        assert api.ddl_wait_all(world.id) == 0
    finally:
        lib.ddl_set_config(b'pipeline_rounds', 1)
    assert len(order) == uid and all(s == 0 for s in statuses)
    torch.cuda.synchronize()
    for w, o in want.values():
        assert torch.equal(o, w)


def test_keyed_rounds_pipelined_done_order(world, lib, data_plane_at_one_rank):
    """done() across pipelined rounds in submission order: single-request submits, each its own
    user value, keys sorting in submission order; batches of requests registered while earlier
    rounds are still on the device."""
    from ddl.torch import cpp_backend as cb
    from ddl.torch.util import ddl_dtype
    order, statuses = [], []

    @cb.DONE_FN
    def done(status, user):
        statuses.append(status)
        order.append(user)

    api = cb.CPPBackend.c_api()
    stream = torch.cuda.current_stream()
    keep = []
    n = 400
    for i in range(n):
        t = torch.full((int(1 + (i * 7919) % 300_000),), float(i), device='cuda')
        keep.append(t)
        assert api.ddl_allreduce_submit(world.id, f'ord{i:05d}'.encode(), t.data_ptr(), t.data_ptr(), t.numel(),
                                        ddl_dtype(t), 0, stream.cuda_stream, done, i + 1) == 0
    assert api.ddl_wait_all(world.id) == 0
    assert order == list(range(1, n + 1)) and set(statuses) == {0}
    torch.cuda.synchronize()
    for i, t in enumerate(keep):
        assert bool((t == float(i)).all())


def test_dp_optimizer_wrapper_size1(world):
    from ddl.torch.parallelism.data import data_parallelism_distributed_optimizer_wrapper
    torch.manual_seed(0)
    m = torch.nn.Linear(16, 4).cuda()
    ref = torch.nn.Linear(16, 4).cuda()
    ref.load_state_dict(m.state_dict())
    opt = data_parallelism_distributed_optimizer_wrapper(torch.optim.SGD(m.parameters(), lr=0.1), world)
    ref_opt = torch.optim.SGD(ref.parameters(), lr=0.1)
    assert opt.is_distributed_optimizer and isinstance(opt, torch.optim.SGD)
    x = torch.randn(8, 16, device='cuda')
    for mod, o in ((m, opt), (ref, ref_opt)):
        o.zero_grad()
        mod(x).square().sum().backward()
        o.step()
    for a, b in zip(m.parameters(), ref.parameters()):
        assert torch.equal(a, b)


def test_split_size1(world):
    sub = world.split_communicator(0)
    assert sub.size == 1 and sub.rank == 0
    from ddl.torch.tensor_communicate import allreduce
    x = torch.arange(10.0, device='cuda')
    assert torch.equal(allreduce(x, sub), x)
    sub.detach()


def test_split_size1_keyed_detach_joins_handler(world):
    """A size-1 split that ran keyed requests starts a request handler (two threads); detach must
    destroy the split and join them. r05's soak found rank 4 at P = 5 (a size-1 pair) gaining two
    threads per round: the handler held an owning pointer to its own communicator, a cycle."""
    from ddl.torch.tensor_communicate import allreduce_async_batch

    def keyed_round(i):
        sub = world.split_communicator(0)
        xs = [torch.full((100 + j,), float(i + j), device='cuda') for j in range(3)]
        for hd, x in zip(allreduce_async_batch(xs, [f'leak_{j}' for j in range(3)], sub), xs):
            assert torch.equal(hd.wait(timeout=60), x)
        sub.detach()

    def threads():
        gc.collect()
        return len(os.listdir('/proc/self/task'))

    keyed_round(0)  # lazily started pools / threads settle first
    n0 = threads()
    for i in range(1, 6):
        keyed_round(i)
    assert threads() <= n0 + 1, (n0, threads())


def test_done_callback_may_detach_its_communicator(world):
    """A done() that detaches its own communicator drops the last reference on the handler's
    completion thread, and ~RequestHandler joins that thread: the engine hands the destruction to
    a thread of its own (engine.h, CommunicatorDeleter). The process survives, the callback's
    detach returns, and the handler's threads end."""
    import time

    from ddl.torch import cpp_backend as cb
    from ddl.torch.util import ddl_dtype
    api = cb.CPPBackend.c_api()
    sub = world.split_communicator(0)
    seen = []

    @cb.DONE_FN
    def done(status, user):
        seen.append(status)
        api.detach_communicator(sub.id)
        seen.append('detached')

    n0 = len(os.listdir('/proc/self/task'))  # before the split's handler starts (lazily)
    t = torch.ones(64, device='cuda')
    assert api.ddl_allreduce_submit(sub.id, b'detach_me', t.data_ptr(), t.data_ptr(), 64, ddl_dtype(t), 0,
                                    torch.cuda.current_stream().cuda_stream, done, 0) == 0
    deadline = time.time() + 30
    while time.time() < deadline and (len(seen) < 2 or len(os.listdir('/proc/self/task')) > n0):
        time.sleep(0.05)
    assert seen == [0, 'detached'], seen
    assert len(os.listdir('/proc/self/task')) <= n0
    assert api.communicator_size(sub.id) == -1  # gone from the registry


def test_rccl_comparator_entry_size1(world, lib):
    x = torch.randn(1000, device='cuda')
    y = torch.empty_like(x)
    assert lib.ddl_allreduce_variant(world.id, x.data_ptr(), y.data_ptr(), 1000, 1, 0,
                                     torch.cuda.current_stream().cuda_stream, 1) == 0
    torch.cuda.synchronize()
    assert torch.equal(x, y)


@pytest.fixture
def data_plane_at_one_rank(lib):
    """Runs the keyed data plane (pack -> allreduce -> unpack) in the one-rank world instead of
    the shortcut, so the fusion path's composition is exercised on one GPU."""
    keys = (b'one_rank_shortcut', b'fusion_pipeline_bytes', b'fusion_threshold_bytes')
    old = {k: lib.ddl_get_config(k) for k in keys}
    assert lib.ddl_set_config(b'one_rank_shortcut', 0) == 0
    yield
    for k, v in old.items():
        assert lib.ddl_set_config(k, v) == 0


@pytest.mark.parametrize('pipeline', [0, 256, 4096, 1 << 20, 256 << 20])
@pytest.mark.parametrize('threshold', [(1 << 31) - 1, 3 << 20])
def test_keyed_fusion_pipeline_data_plane(world, lib, data_plane_at_one_rank, pipeline, threshold):
    """Multi-request plans through pack -> allreduce -> unpack, pipelined over sub-plans of at
    most `pipeline` bytes (segments cut at 256-byte multiples; two fusion buffers; pack/unpack
    on a side stream), plans capped at `threshold`: every output equals its input (P = 1), in
    place and out of place, for every dtype and ragged sizes."""
    from ddl.torch.tensor_communicate import allreduce_async_batch
    assert lib.ddl_set_config(b'fusion_pipeline_bytes', pipeline) == 0
    assert lib.ddl_set_config(b'fusion_threshold_bytes', threshold) == 0
    rng = np.random.default_rng(pipeline ^ threshold)
    dts = [torch.float32, torch.float16, torch.int32, torch.bfloat16, torch.float64, torch.int64]
    tensors, names, outputs = [], [], []
    for i in rng.permutation(150):
        n = int(np.exp(rng.uniform(0, np.log(300_000))))
        dt = dts[i % len(dts)]
        t = (torch.randn(n, device='cuda') * 1000).to(dt)
        tensors.append(t)
        names.append(f'pipe_{i:04d}')
        outputs.append(t if i % 3 == 0 else torch.full_like(t, 7))
    want = [t.clone() for t in tensors]
    hs = allreduce_async_batch(tensors, names, world, outputs=outputs)
    for w, h in zip(want, hs):
        got = h.wait(timeout=60)
        assert torch.equal(got, w)


def test_keyed_fusion_pipeline_large_segment(world, lib, data_plane_at_one_rank):
    """One segment larger than several sub-plans next to small ones: the big tensor is cut
    across sub-plans and both fusion buffers are reused many times."""
    from ddl.torch.tensor_communicate import allreduce_async_batch
    assert lib.ddl_set_config(b'fusion_pipeline_bytes', 1 << 20) == 0
    big = torch.randn(5_000_003, device='cuda')
    small = [torch.randn(k, device='cuda') for k in (1, 17, 4099)]
    ts = [small[0], big, small[1], small[2]]
    want = [t.clone() for t in ts]
    hs = allreduce_async_batch(ts, ['a', 'b', 'c', 'd'], world)
    for w, h in zip(want, hs):
        assert torch.equal(h.wait(timeout=60), w)


@pytest.mark.parametrize('memory', ['pageable', 'pinned', 'pinned_outputs', 'mixed', 'pinned_misaligned',
                                    'registered'])
@pytest.mark.parametrize('chunk', [4096, 64 << 10, 32 << 20])
def test_keyed_host_requests_data_plane(world, lib, chunk, memory):
    """Keyed requests on host tensors with the one-rank shortcut off: every plan goes through the
    host pipeline in chunks (4096 B chunks make hundreds of chunks over 4 slots), in and out of
    place, every dtype, plus a device request in the same batch; outputs equal the inputs bit for
    bit (one rank). Pageable outputs are staged back (D2H -> host unpack); when every output of a
    plan is pinned the unpack kernel writes them over PCIe — the plan counter says which path
    ran. A pinned output viewed at a 2-byte offset, or one pageable output in the dtype group,
    sends its plan back to staging. 'registered': pageable tensors with the opt-in
    registration cache take the pinned paths (the unpack kernel writes the registered outputs
    through their device mapping); switching the cache off unregisters them again."""
    from ddl.torch.tensor_communicate import allreduce_async_batch, broadcast_async
    keys = (b'one_rank_shortcut', b'host_chunk_bytes', b'host_register_cache_bytes')
    old = {k: lib.ddl_get_config(k) for k in keys}
    try:
        assert lib.ddl_set_config(b'one_rank_shortcut', 0) == 0
        assert lib.ddl_set_config(b'host_chunk_bytes', chunk) == 0
        if memory == 'registered':
            assert lib.ddl_set_config(b'host_register_cache_bytes', 1 << 30) == 0
        g = torch.Generator().manual_seed(chunk)
        dts = [torch.float32, torch.float64, torch.int32, torch.float16, torch.bfloat16, torch.int64]
        xs = [(torch.randn(n, generator=g) * 100).to(dts[i % 6]) for i, n in enumerate([1, 7, 1000, 65_537, 300_001,
                                                                                       5, 2_000_003, 4096])]
        if memory in ('pinned', 'mixed', 'pinned_misaligned'):
            xs = [x.pin_memory() for x in xs]
        if memory == 'pinned_misaligned':  # fp16 tensor 3 (in place) seen from its second element: 2-byte offset
            xs[3] = xs[3][1:]
        keep = [x.clone() for x in xs]
        # odd tensors in place, even ones into fresh outputs (int32 tensor 2: pageable when mixed)
        outs = [x if i % 2 else torch.empty_like(x, pin_memory=memory not in ('pageable', 'registered') and
                                                 (memory, i) != ('mixed', 2))
                for i, x in enumerate(xs)]
        if memory == 'pinned_outputs':  # pageable inputs, every output pinned
            outs = [torch.empty_like(x, pin_memory=True) for x in xs]
        dev = torch.randn(1234, device='cuda')
        plans0 = lib.ddl_get_config(b'host_zero_copy_plans')
        tl_keys = (b'host_pack_us', b'host_wait_us', b'host_unpack_us')
        tl0 = [lib.ddl_get_config(k) for k in tl_keys]
        hs = allreduce_async_batch(xs + [dev], [f'hk_{i}' for i in range(len(xs))] + ['hk_dev'], world,
                                   outputs=outs + [torch.empty_like(dev)])
        for h, k in zip(hs, keep):
            got = h.wait(timeout=60)
            assert not got.is_cuda and torch.equal(got, k)
        assert torch.equal(hs[-1].wait(timeout=60), dev)
        # one plan per host dtype group (6 dtypes); staged: the mixed int32 group and the
        # misaligned fp16 group
        device_unpacked = lib.ddl_get_config(b'host_zero_copy_plans') - plans0
        assert device_unpacked == {'pageable': 0, 'pinned': 6, 'pinned_outputs': 6, 'mixed': 5,
                                   'pinned_misaligned': 5, 'registered': 6}[memory]
        # the engine thread's timeline statistics moved: chunks were packed, and unpacked on the
        # host when every plan was staged back (microseconds: a tiny staged plan may read 0)
        pack, wait, unpack = [lib.ddl_get_config(k) - v for k, v in zip(tl_keys, tl0)]
        assert pack > 0 and wait >= 0 and unpack >= 0, (pack, wait, unpack)
        assert unpack > 0 or device_unpacked > 0, (memory, unpack)
        t = torch.arange(100_003, dtype=torch.float64)
        assert torch.equal(broadcast_async(t, 'hk_b', 0, world).wait(timeout=60), t)
    finally:
        for k, v in old.items():
            lib.ddl_set_config(k, v)


@pytest.mark.parametrize('zero_copy', [0, 1])
def test_host_plan_failure_drains_unpacks(world, lib, zero_copy):
    """a host plan whose staging loop fails midway — here its collective at
    chunk 8, past the 4 download slots, so unpack jobs of earlier chunks are queued on the unpack
    lane — reports the error only once every unpack already submitted has written its chunk:
    after done(error) the output never changes again (the caller may free it then). Chunks 0-7
    hold the input, the rest is untouched. A failed keyed collective stops its communicator's
    handler by design (later submissions there are refused), so the fault runs on a split
    communicator of its own; the world's handler keeps working. ADVICE r5: also with pinned
    tensors and host_zero_copy 1, where the unpack kernel writes the outputs over PCIe from d2h_ —
    those kernels must have finished before done(error) too."""
    import time

    import _helpers as h
    from ddl.torch.cpp_backend import DDLError
    from ddl.torch.tensor_communicate import allreduce_async
    chunk = 256 << 10
    x = torch.arange(3_000_017, dtype=torch.float32)
    out = torch.full_like(x, -7.0)
    if zero_copy:
        x, out = x.pin_memory(), out.pin_memory()
    plans0 = lib.ddl_get_config(b'host_zero_copy_plans')
    sub = world.split_communicator(0)
    try:
        with h.config(lib, one_rank_shortcut=0, host_chunk_bytes=chunk, host_zero_copy=zero_copy):
            assert lib.ddl_testing_host_coll_fault(8) == 0
            try:
                hd = allreduce_async(x, 'fault_plan', sub, output=out)
                with pytest.raises(DDLError):
                    hd.wait(timeout=60)
                snap = out.clone()
                time.sleep(0.3)
                assert torch.equal(out, snap), 'the output changed after done(error)'
            finally:
                assert lib.ddl_testing_host_coll_fault(-1) == 0
            assert (lib.ddl_get_config(b'host_zero_copy_plans') > plans0) == bool(zero_copy)
            k = 8 * chunk // 4
            assert torch.equal(out[:k], x[:k])
            assert bool((out[k:] == -7.0).all())
            with pytest.raises(DDLError):  # the failed handler refuses further requests
                allreduce_async(x, 'after_fault', sub, output=out).wait(timeout=60)
            y = torch.arange(1_000_003, dtype=torch.float32)
            assert torch.equal(allreduce_async(y, 'world_after_fault', world, output=torch.empty_like(y)).wait(
                timeout=60), y)
    finally:
        sub.detach()


def test_registration_cache_address_reuse(world, lib):
    """the registration cache is keyed by virtual address. r04 measured what the
    advisor feared: a cached pageable range unmapped and mapped afresh at the same address (munmap,
    then mmap MAP_FIXED) and used again faults the GPU (illegal memory access) — the old
    registration's device mapping points at pages that are gone. So a cached range must leave the
    cache before its memory is freed: ddl_host_unregister, which the torch mirror calls from a
    finalizer of every host tensor it submits while the cache is on. Here, three rounds of: a
    tensor over the mapping, two keyed allreduces in place (the second a cache hit through the
    zero-copy unpack), the tensor dropped (its finalizer unregisters the range: registered bytes
    back to where they were), then new pages at the same address — the next round's result is the
    new tensor's, bit for bit. The munmap only happens once the range is out of the cache."""
    import gc
    import mmap as _mmap
    from ddl.torch.tensor_communicate import allreduce_async
    libc = ctypes.CDLL(None, use_errno=True)
    libc.mmap.restype = ctypes.c_void_p
    libc.mmap.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_long]
    libc.munmap.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
    n = 3 << 20  # 12 MiB of fp32: several host chunks below
    size = n * 4
    prot = _mmap.PROT_READ | _mmap.PROT_WRITE
    flags = _mmap.MAP_PRIVATE | _mmap.MAP_ANONYMOUS
    MAP_FIXED = 0x10
    addr = libc.mmap(None, size, prot, flags, -1, 0)
    assert addr not in (None, ctypes.c_void_p(-1).value)
    keys = (b'one_rank_shortcut', b'host_chunk_bytes', b'host_register_cache_bytes', b'host_zero_copy')
    old = {k: lib.ddl_get_config(k) for k in keys}
    try:
        for k, v in ((b'one_rank_shortcut', 0), (b'host_chunk_bytes', 4 << 20), (b'host_register_cache_bytes', 1 << 30),
                     (b'host_zero_copy', 1)):
            assert lib.ddl_set_config(k, v) == 0
        g = torch.Generator().manual_seed(5)
        reg0 = lib.ddl_get_config(b'host_registered_bytes')
        for rnd in range(3):
            x = torch.frombuffer((ctypes.c_char * size).from_address(addr), dtype=torch.float32)
            want = torch.randn(n, generator=g)
            x.copy_(want)
            for call in range(2):
                hits0, zc0 = lib.ddl_get_config(b'host_register_hits'), lib.ddl_get_config(b'host_zero_copy_plans')
                got = allreduce_async(x, f'reuse_{rnd}_{call}', world, output=x).wait(timeout=60)  # in place
                assert torch.equal(got, want), f'round {rnd} call {call}: not the tensor now at the address'
                del got
            # the second call found the range in the cache and unpacked on the device
            assert lib.ddl_get_config(b'host_register_hits') > hits0
            assert lib.ddl_get_config(b'host_zero_copy_plans') > zc0
            assert lib.ddl_get_config(b'host_registered_bytes') >= reg0 + size
            unreg0 = lib.ddl_get_config(b'host_unregistered_ranges')
            del x
            gc.collect()
            # the tensor's finalizer took the range out of the cache: safe to free it now
            assert lib.ddl_get_config(b'host_unregistered_ranges') > unreg0
            assert lib.ddl_get_config(b'host_registered_bytes') == reg0
            assert libc.munmap(ctypes.c_void_p(addr), size) == 0
            again = libc.mmap(ctypes.c_void_p(addr), size, prot, flags | MAP_FIXED, -1, 0)
            assert again == addr
        # the C-ABI contract directly: a cached range, ddl_host_unregister, the cache no longer holds it
        y = torch.frombuffer((ctypes.c_char * size).from_address(addr), dtype=torch.float32)
        y.fill_(2.0)
        assert torch.equal(allreduce_async(y, 'reuse_c', world, output=y).wait(timeout=60), torch.full((n,), 2.0))
        assert lib.ddl_get_config(b'host_registered_bytes') >= reg0 + size
        assert lib.ddl_host_unregister(ctypes.c_void_p(addr), ctypes.c_size_t(size)) == 0
        assert lib.ddl_get_config(b'host_registered_bytes') == reg0
        del y
        gc.collect()
    finally:
        assert lib.ddl_set_config(b'host_register_cache_bytes', 0) == 0  # unregisters the cached range
        for k, v in old.items():
            lib.ddl_set_config(k, v)
        libc.munmap(ctypes.c_void_p(addr), size)


def _cpulist(text):
    out = set()
    for part in text.strip().split(','):
        if part:
            a, _, b = part.partition('-')
            out.update(range(int(a), int(b or a) + 1))
    return out


def test_host_threads_bound_to_gpu_numa_node(world, lib):
    """config host_numa_bind (default on): after a keyed host plan, the handler's engine thread and
    copy threads run on the CPUs of the GPU's NUMA node (within the process's affinity) — where
    HIP places pinned host memory. Skipped where that would not narrow the set."""
    import glob
    import os
    from ddl.torch.tensor_communicate import allreduce_async_batch
    p = torch.cuda.get_device_properties(0)
    bdf = f'{getattr(p, "pci_domain_id", 0):04x}:{getattr(p, "pci_bus_id", 0):02x}:{getattr(p, "pci_device_id", 0):02x}.0'
    try:
        node = int(open(f'/sys/bus/pci/devices/{bdf}/numa_node').read())
        local = _cpulist(open(f'/sys/devices/system/node/node{node}/cpulist').read())
    except (OSError, ValueError):
        pytest.skip('no NUMA information for the GPU')
    allowed = os.sched_getaffinity(0)
    want = local & allowed
    if node < 0 or not want or want == allowed:
        pytest.skip('binding would not narrow the CPU set here')
    assert lib.ddl_get_config(b'host_numa_bind') == 1
    old = lib.ddl_get_config(b'one_rank_shortcut')
    try:
        assert lib.ddl_set_config(b'one_rank_shortcut', 0) == 0
        xs = [torch.randn(300_001) for _ in range(3)]  # host tensors: the copy threads run
        for h in allreduce_async_batch(xs, [f'numa_{i}' for i in range(3)], world):
            h.wait(timeout=60)
    finally:
        lib.ddl_set_config(b'one_rank_shortcut', old)
    bound = 0
    for st in glob.glob(f'/proc/{os.getpid()}/task/*/status'):
        try:
            line = [x for x in open(st) if x.startswith('Cpus_allowed_list:')][0]
        except (OSError, IndexError):
            continue
        if _cpulist(line.split(':', 1)[1]) == want:
            bound += 1
    # the engine thread, plus the copy threads (host_copy_threads, default 7)
    assert bound >= 1 + lib.ddl_get_config(b'host_copy_threads'), (bound, sorted(want)[:4])
