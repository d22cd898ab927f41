"""Worker of tests/test_multiproc_gpu.py: P processes share the one GPU and run the whole engine
as at N > 1 — world communicator, TCP token ring, keyed handler, fusion pipeline, ring / direct /
one-shot schedules, the autotuner, streams and kernels — with only the point-to-point groups
carried differently: through gloo on host copies (ddl_init_test_transport), because RCCL
refuses two ranks of one host on one device — or, with transport='rccl', over real multi-rank RCCL
(rccl_sockets_env). Every check compares with the oracle or an exact sum; every
rank runs the same checks in the same order (they are collectives) and reports
(name, ok, detail). Test infrastructure only."""
import contextlib
import ctypes
import os
import sys
import traceback

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)


# ---- checks ------------------------------------------------------------------------------------
def _dev(torch, x, dev):
    return torch.from_numpy(x.view(np.int16) if x.dtype == np.uint16 else x).to(dev)


def _host(t, like):
    return t.cpu().numpy().view(like.dtype)


def check_reference_known_answers(ctx):
    """The reference's own test scripts (src/py/ddl/test/*.py) with their known answers."""
    torch, comm, P, r = ctx['torch'], ctx['comm'], ctx['P'], ctx['rank']
    from ddl.torch.tensor_communicate import allgather, allreduce, broadcast
    x = torch.full((16,), float(r), device='cuda')  # allreduce_test.py:13
    assert torch.equal(allreduce(x, comm), torch.full((16,), float(P * (P - 1) // 2), device='cuda'))
    root = 3 if P >= 4 else P - 1  # broadcast_test.py:13-14 (root 3 needs P >= 4)
    y = torch.full((16,), float(r + 1), device='cuda')
    assert torch.equal(broadcast(y, root, comm), torch.full((16,), float(root + 1), device='cuda'))
    v = torch.arange(4 + r, dtype=torch.float32, device='cuda') + r  # allgather_test.py:13-21
    idx = torch.tensor([[0, 0], [1, 1], [2, 2], [3, 3]], dtype=torch.float32, device='cuda') + r
    want_v = torch.cat([torch.arange(4 + q, dtype=torch.float32) + q for q in range(P)])
    want_i = torch.cat([torch.tensor([[0, 0], [1, 1], [2, 2], [3, 3]], dtype=torch.float32) + q for q in range(P)])
    assert torch.equal(allgather(v, comm).cpu(), want_v)
    assert torch.equal(allgather(idx, comm).cpu(), want_i)


def check_schedules_vs_oracle(ctx):
    """ddl_allreduce with each schedule fixed (tuner off): every rank equals the oracle's
    summation in that schedule's order, bit for bit, in and out of place, all dtypes — with
    reference_order 1 (default) MPICH's own order whatever the schedule, with 0 the ring /
    left-fold orders."""
    import _helpers as h
    torch, lib, comm, P, r, ora = ctx['torch'], ctx['lib'], ctx['comm'], ctx['P'], ctx['rank'], ctx['oracle']
    s = torch.cuda.current_stream().cuda_stream
    cases = [(algo, ref) for ref in (1, 0) for algo in (0, 1, 2, 3)]
    with h.config(lib, tune=0, slice_bytes=64 << 10):
        for algo, ref in cases:
            with h.config(lib, algo=algo, reference_order=ref):
                for dt in (h.DT_FLOAT, h.DT_HALF, h.DT_INT32, h.DT_BFLOAT16, h.DT_DOUBLE):
                    for n in ((1, 300, 4099, 300_001) if ref else (1, 4099, 300_001)):
                        xs = [h.random_input(dt, n, 100 * algo + 7 * dt + 13 * q + n) for q in range(P)]
                        if ref:
                            want = ora.fold_ref_order(dt, xs)
                        elif algo == 0:
                            R, _ = h.ring_shape(lib, n, dt, P)
                            want = ora.allreduce_ring(dt, xs, h.ring_perms(lib, P, R))
                        elif algo == 1:
                            want = ora.allreduce_direct(dt, xs)
                        else:  # one-shot / gather-fold: left fold in rank order
                            want = ora.fold(dt, xs)
                        for in_place in (False, True):
                            a = _dev(torch, xs[r], 'cuda')
                            b = a if in_place else torch.empty_like(a)
                            st = lib.ddl_allreduce(comm.id, a.data_ptr(), b.data_ptr(), n, dt, 0, s)
                            assert st == 0, lib.ddl_last_error()
                            got = _host(b, xs[r])
                            assert got.tobytes() == want.tobytes(), (algo, ref, dt, n, in_place)


def check_allreduce_batch(ctx):
    """The grouped allreduce on the real engine (Communicator::allreduce_batch through the
    allreduce_batch_ Python API): mixed bucket sizes (empty, ragged, both sides of 2048 B) of fp32
    and fp16, the direct and one-shot schedules and the tuner's pick — every bucket on every rank
    equals MPICH's order for its own message, bit for bit."""
    import _helpers as h
    torch, lib, comm, P, r, ora = ctx['torch'], ctx['lib'], ctx['comm'], ctx['P'], ctx['rank'], ctx['oracle']
    from ddl.torch.tensor_communicate import allreduce_batch_
    ns = [300, 0, 4099, 65_537, 1, 300_001]
    for dt in (h.DT_FLOAT, h.DT_HALF):
        for settings in ({'tune': 0, 'algo': 1, 'slice_bytes': 64 << 10}, {'tune': 0, 'algo': 2}, {}):
            xs = [[h.random_input(dt, n, 1000 * q + 17 * b + dt) for b, n in enumerate(ns)] for q in range(P)]
            ts = [_dev(torch, x.view(np.uint16) if x.dtype == np.float16 else x, 'cuda') for x in xs[r]]
            ts = [t.view(torch.float16) if dt == h.DT_HALF else t for t in ts]
            with h.config(lib, **settings):
                allreduce_batch_(ts, comm)
            torch.cuda.synchronize()
            for b, n in enumerate(ns):
                if n:
                    want = ora.fold_ref_order(dt, [xs[q][b] for q in range(P)])
                    got = ts[b].view(torch.int16).cpu().numpy().view(np.float16) if dt == h.DT_HALF else ts[b].cpu().numpy()
                    assert got.tobytes() == want.tobytes(), (dt, settings, b, n)


def check_tuned_exact(ctx):
    """Autotuner on (collective timing, max over ranks through the transport): every rank picks
    the same schedule per size class, and exactly summable buckets come out exact."""
    import _helpers as h
    torch, lib, comm, P, r, dist = ctx['torch'], ctx['lib'], ctx['comm'], ctx['P'], ctx['rank'], ctx['dist']
    s = torch.cuda.current_stream().cuda_stream
    with h.config(lib, tune=1):
        picks = []
        for nbytes in (64 << 10, 4 << 20, 24 << 20 if P < 8 else 8 << 20):
            n = nbytes // 4
            xs = [h.random_input(h.DT_FLOAT, n, 5 + q, kind='exact') for q in range(P)]
            want = np.sum(np.stack(xs).astype(np.float64), axis=0).astype(np.float32)
            a = _dev(torch, xs[r], 'cuda')
            assert lib.ddl_allreduce(comm.id, a.data_ptr(), a.data_ptr(), n, h.DT_FLOAT, 0, s) == 0, lib.ddl_last_error()
            assert np.array_equal(_host(a, xs[r]), want), nbytes
            chosen, count = ctypes.c_int(-1), ctypes.c_int(0)
            cfgs = (ctypes.c_longlong * 64)()
            tms = (ctypes.c_float * 16)()
            assert lib.ddl_tune_result(comm.id, nbytes, ctypes.byref(chosen), ctypes.byref(count), cfgs, tms, 16) == 0
            assert chosen.value >= 0 and count.value >= 2
            picks.append((chosen.value, [round(tms[i], 6) for i in range(count.value)]))
        everyone = [None] * P
        dist.all_gather_object(everyone, picks)
        assert all(e == picks for e in everyone), everyone  # same choice and same agreed times


def check_keyed_fusion(ctx):
    """Keyed batches registered in a different order on every rank: negotiated, grouped by dtype,
    fused into plans capped at 1 MiB + 1 and pipelined over 256 KiB sub-plans; two rounds (the
    second by id-table index). Integer-valued data, so every dtype's sum is exact."""
    import _helpers as h
    torch, lib, comm, P, r = ctx['torch'], ctx['lib'], ctx['comm'], ctx['P'], ctx['rank']
    from ddl.torch.tensor_communicate import allreduce_async_batch
    dts = [torch.float32, torch.float16, torch.int32, torch.bfloat16, torch.float64, torch.int64]
    rng = np.random.default_rng(11)
    k = 120
    sizes = [int(np.exp(rng.uniform(0, np.log(200_000)))) for _ in range(k)]
    with h.config(lib, fusion_threshold_bytes=(1 << 20) + 1, fusion_pipeline_bytes=256 << 10):
        for rnd in range(2):
            gen = [torch.Generator().manual_seed(1000 * rnd + i) for i in range(k)]
            base = [torch.randint(-8, 9, (sizes[i],), generator=gen[i]) for i in range(k)]
            ts = [(base[i] + r).to(dts[i % len(dts)]).cuda() for i in range(k)]
            want = [(base[i] * P + P * (P - 1) // 2).to(dts[i % len(dts)]) for i in range(k)]
            order = np.random.default_rng(100 * rnd + r).permutation(k)  # per-rank submission order
            hs = allreduce_async_batch([ts[i] for i in order], [f'g_{i:04d}' for i in order], comm)  # same keys
            for i, hd in zip(order, hs):
                got = hd.wait(timeout=120).cpu()
                assert torch.equal(got, want[i]), (rnd, i, dts[i % len(dts)])
    sr, cr = ctypes.c_longlong(), ctypes.c_longlong()
    assert lib.ddl_control_stats(ctypes.byref(sr), ctypes.byref(cr)) == 0
    assert cr.value >= 1  # the repeated key set went by id-table index


def check_keyed_reference_order(ctx):
    """Random fp32 / fp64 gradients (not exactly summable) through the keyed path — negotiated,
    fused per dtype into one plan, pipelined over 256 KiB sub-plans: every element equals
    MPICH's order for the plan's message (ddlo_fold_ref_order with the group's bytes), bit for
    bit, on every rank (reference_order default)."""
    import _helpers as h
    torch, lib, comm, P, r, ora = ctx['torch'], ctx['lib'], ctx['comm'], ctx['P'], ctx['rank'], ctx['oracle']
    from ddl.torch.tensor_communicate import allreduce_async_batch
    sizes = [5, 300, 70_001, 4099, 1, 200_000, 513]
    dts = [h.DT_FLOAT if i % 2 == 0 else h.DT_DOUBLE for i in range(len(sizes))]
    xs = [[h.random_input(dts[i], n, 500 + 31 * i + q) for q in range(P)] for i, n in enumerate(sizes)]
    group_bytes = {d: sum(xs[i][0].nbytes for i in range(len(sizes)) if dts[i] == d) for d in set(dts)}
    with h.config(lib, fusion_pipeline_bytes=256 << 10, reference_order=1):
        ts = [torch.from_numpy(xs[i][r]).cuda() for i in range(len(sizes))]
        hs = allreduce_async_batch(ts, [f'ro_{i:02d}' for i in range(len(sizes))], comm)
        for i, hd in enumerate(hs):
            got = hd.wait(timeout=120).cpu().numpy()
            want = ora.fold_ref_order(dts[i], xs[i], group_bytes[dts[i]])
            assert got.tobytes() == want.tobytes(), (i, sizes[i])


def check_split_communicators_keyed(ctx):
    """One token ring and handler per communicator (RingTokenCommunicateController.cc:53-79):
    keyed batches run at once on the world, on pairs {0,1}, {2,3}, ... (color rank // 2) and on a
    same-size split with reversed keys, all under the SAME key names and submitted in per-rank
    random orders. Each output equals MPICH's order over that communicator's ranks
    (ddlo_fold_ref_order with the dtype group's bytes) — no cross-talk between rings. Then plain
    allreduces on the splits (rank mapping of the data plane) with the autotuner on."""
    import _helpers as h
    torch, lib, comm, P, r, ora = ctx['torch'], ctx['lib'], ctx['comm'], ctx['P'], ctx['rank'], ctx['oracle']
    from ddl.torch.tensor_communicate import allreduce, allreduce_async_batch
    pair = comm.split_communicator(r // 2, r)
    same = comm.split_communicator(0, P - 1 - r)
    members = {'world': list(range(P)), 'pair': [q for q in range(P) if q // 2 == r // 2],
               'same': list(range(P - 1, -1, -1))}
    assert (pair.size, pair.rank) == (len(members['pair']), members['pair'].index(r))
    assert (same.size, same.rank) == (P, P - 1 - r)
    comms = {'world': comm, 'pair': pair, 'same': same}
    sizes = [7, 300, 5000, 70_001, 1, 4099]
    dts = [h.DT_FLOAT, h.DT_INT32, h.DT_FLOAT, h.DT_DOUBLE, h.DT_FLOAT, h.DT_INT32]
    # over real RCCL, keyed rounds of two SPLITS that share ranks can meet on one in-order
    # hardware queue (both in the least priority's pool, config queue_isolation) in different
    # orders on different ranks: the world's rounds run beside the pair's, the
    # same-size split's after them (queue_isolation 0: one communicator at a time);
    # DDL_MP_CONCURRENT_SPLITS=1 runs all three at once
    flush_before = set()
    if ctx.get('transport') == 'rccl' and os.environ.get('DDL_MP_CONCURRENT_SPLITS') != '1':
        flush_before = {'same'} if lib.ddl_get_config(b'queue_isolation') == 1 else {'pair', 'same'}
    for rnd in range(2):  # the second round goes by id-table index on every ring
        handles, wants = [], []
        for ci, (name, c) in enumerate(comms.items()):
            if name in flush_before and handles:
                for hd, (nm, i, want) in zip(handles, wants):
                    assert hd.wait(timeout=120).cpu().numpy().tobytes() == want.tobytes(), (rnd, nm, i)
                handles, wants = [], []
            xs = [[h.random_input(dts[i], n, 1000 * rnd + 100 * ci + 31 * i + q) for q in range(P)]
                  for i, n in enumerate(sizes)]
            mem = members[name]
            gb = {d: sum(xs[i][0].nbytes for i in range(len(sizes)) if dts[i] == d) for d in set(dts)}
            order = np.random.default_rng(7 * rnd + 13 * ci + r).permutation(len(sizes))
            ts = [torch.from_numpy(xs[i][r]).cuda() for i in order]
            handles += allreduce_async_batch(ts, [f'k_{i}' for i in order], c)
            wants += [(name, i, ora.fold_ref_order(dts[i], [xs[i][q] for q in mem], gb[dts[i]])) for i in order]
        for hd, (name, i, want) in zip(handles, wants):
            got = hd.wait(timeout=120).cpu().numpy()
            assert got.tobytes() == want.tobytes(), (rnd, name, i)
    with h.config(lib, tune=1):
        for name in ('pair', 'same'):
            c = comms[name]
            n = 1 << 18
            xs = [h.random_input(h.DT_FLOAT, n, 77 + q, kind='exact') for q in range(P)]
            got = allreduce(torch.from_numpy(xs[r]).cuda(), c).cpu().numpy()
            want = np.sum(np.stack([xs[q] for q in members[name]]).astype(np.float64), axis=0).astype(np.float32)
            assert np.array_equal(got, want), name
    pair.detach()
    same.detach()


def check_queue_classes(ctx):
    """Config queue_isolation: with it on, over RCCL the world's executor streams sit
    at the default priority, its keyed data plane (handler stream, private communicator) at the
    greatest and a split's streams at the least — three pools of HIP's in-order hardware queues;
    with the key at 0 (default), or over the test transport (no RCCL kernels), every stream at the
    default. A keyed
    batch on the split and on the world stays bit-exact vs MPICH's order."""
    import _helpers as h
    torch, lib, comm, P, r, ora = ctx['torch'], ctx['lib'], ctx['comm'], ctx['P'], ctx['rank'], ctx['oracle']
    from ddl.torch.tensor_communicate import allreduce_async_batch
    rccl = ctx.get('transport') == 'rccl'

    def prios(c):
        out = (ctypes.c_int * 4)()
        assert lib.ddl_testing_stream_priorities(ctypes.c_longlong(c.id), out) == 0, lib.ddl_last_error()
        return list(out)

    def keyed(c, tag):
        xs = [[h.random_input(h.DT_FLOAT, 3000 + 7 * i, 400 + 10 * i + q) for q in range(P)] for i in range(2)]
        hs = allreduce_async_batch([torch.from_numpy(x[r]).cuda() for x in xs], [f'{tag}_a', f'{tag}_b'], c)
        gb = sum(x[0].nbytes for x in xs)
        for hd, x in zip(hs, xs):
            assert hd.wait(timeout=120).cpu().numpy().tobytes() == ora.fold_ref_order(h.DT_FLOAT, x, gb).tobytes()

    # HIP's range on gfx950 is least 1, greatest -1, default 0 (torch's Stream.priority_range
    # reports (0, -1): it clamps the least to the default), so: more urgent < 0 < less urgent
    keyed(comm, 'qc_world')
    w = prios(comm)  # the world's class was fixed at ddl_init (default 0, DDL_QUEUE_ISOLATION)
    assert w[:2] == [0, 0] and w[2] == w[3] and (w[2] < 0 if rccl and ctx['queue_isolation'] else w[2] == 0), w
    for iso in (1, 0):
        with h.config(lib, queue_isolation=iso):
            sub = comm.split_communicator(0, r)
        try:
            keyed(sub, f'qc_split{iso}')
            p = prios(sub)
            assert len(set(p)) == 1 and (p[0] > 0 if rccl and iso else p[0] == 0), (iso, p)
        finally:
            sub.detach()


def check_rccl_channel_bounds(ctx):
    """Config rccl_min_ctas / rccl_max_ctas: a split created under channel
    bounds (over RCCL: ncclCommSplit with ncclConfig_t.minCTAs / maxCTAs; the test transport ignores
    them) carries the default schedule and a keyed batch bit-exact vs MPICH's order, for two
    settings; the world keeps working after the bounds are restored."""
    import _helpers as h
    torch, lib, comm, P, r, ora = ctx['torch'], ctx['lib'], ctx['comm'], ctx['P'], ctx['rank'], ctx['oracle']
    from ddl.torch.tensor_communicate import allreduce, allreduce_async_batch
    for lo, hi in ((2, 2), (8, 16)):
        with h.config(lib, rccl_min_ctas=lo, rccl_max_ctas=hi):
            sub = comm.split_communicator(0, r)
        try:
            for n in (1000, 300_001):
                xs = [h.random_input(h.DT_FLOAT, n, 555 + 7 * lo + q + n) for q in range(P)]
                got = allreduce(torch.from_numpy(xs[r]).cuda(), sub).cpu().numpy()
                assert got.tobytes() == ora.fold_ref_order(h.DT_FLOAT, xs).tobytes(), (lo, hi, n)
            xs = [[h.random_input(h.DT_DOUBLE, 5000 + i, 90 + 10 * i + q) for q in range(P)] for i in range(3)]
            hs = allreduce_async_batch([torch.from_numpy(x[r]).cuda() for x in xs], ['cta_a', 'cta_b', 'cta_c'], sub)
            gb = sum(x[0].nbytes for x in xs)
            for hd, x in zip(hs, xs):
                assert hd.wait(timeout=120).cpu().numpy().tobytes() == ora.fold_ref_order(h.DT_DOUBLE, x, gb).tobytes()
        finally:
            sub.detach()
    x = torch.full((16,), float(r), device='cuda')
    assert torch.equal(allreduce(x, comm), torch.full((16,), float(P * (P - 1) // 2), device='cuda'))


def check_keyed_host_requests(ctx):
    """Keyed requests on host (CPU) tensors — the reference's only kind (its op is DEVICE_CPU,
    AllreduceOp.cc:68): fused per dtype, staged through pinned 64 KiB chunks (many chunks, the
    4 slots wrap), reduced on the GPU and unpacked back. Every element equals MPICH's order
    for the host group's message (ddlo_fold_ref_order with the group's bytes), bit for bit. A
    device request of the same dtype in the same batch forms its own group. Rounds 2 and 3 pin
    the tensors — on even ranks only (the unpack kernel writes the outputs over PCIe there, D2H
    and host unpack elsewhere: the ranks must still cut the same chunks), then on every rank. Then keyed host broadcasts
    (mixed roots) and allgathers (per-rank first dims)."""
    import _helpers as h
    torch, lib, comm, P, r, ora = ctx['torch'], ctx['lib'], ctx['comm'], ctx['P'], ctx['rank'], ctx['oracle']
    from ddl.torch.tensor_communicate import allgather_async, allreduce_async_batch, broadcast_async
    sizes = [5, 300, 70_001, 4099, 1, 200_000, 513, 33_333]
    dts = [h.DT_FLOAT, h.DT_DOUBLE, h.DT_INT32, h.DT_FLOAT, h.DT_FLOAT, h.DT_DOUBLE, h.DT_INT32, h.DT_FLOAT]
    xs = [[h.random_input(dts[i], n, 900 + 31 * i + q) for q in range(P)] for i, n in enumerate(sizes)]
    gb = {d: sum(xs[i][0].nbytes for i in range(len(sizes)) if dts[i] == d) for d in set(dts)}
    dev_x = [h.random_input(h.DT_FLOAT, 4099, 4000 + q) for q in range(P)]
    for chunk in (64 << 10,):  # many chunks: the 4 upload / download slots wrap
        with h.config(lib, host_chunk_bytes=chunk, reference_order=1):
            for rnd in range(4):
                pin = rnd == 3 or (rnd == 2 and r % 2 == 0)
                ts = [torch.from_numpy(xs[i][r].copy()) for i in range(len(sizes))]
                if pin:
                    ts = [t.pin_memory() for t in ts]
                order = np.random.default_rng(5 * rnd + r).permutation(len(sizes))
                tensors = [ts[i] for i in order] + [torch.from_numpy(dev_x[r]).cuda()]
                names = [f'host_{i}' for i in order] + ['dev_0']
                outs = [t if (rnd % 2 == 1 and not t.is_cuda) else None for t in tensors]  # odd rounds: in place
                plans0 = lib.ddl_get_config(b'host_zero_copy_plans')
                hs = allreduce_async_batch(tensors, names, comm,
                                           outputs=[o if o is not None else torch.empty_like(t, pin_memory=pin and not t.is_cuda)
                                                    for o, t in zip(outs, tensors)])
                for hd, i in zip(hs, order):
                    got = hd.wait(timeout=120)
                    assert not got.is_cuda
                    want = ora.fold_ref_order(dts[i], xs[i], gb[dts[i]])
                    assert got.numpy().tobytes() == want.tobytes(), (rnd, i)
                assert hs[-1].wait(timeout=120).cpu().numpy().tobytes() == ora.fold_ref_order(h.DT_FLOAT, dev_x).tobytes()
                # three host dtype groups, one plan each
                assert lib.ddl_get_config(b'host_zero_copy_plans') - plans0 == (3 if pin else 0), rnd
        hs, want = [], []
        for i in range(9):
            root, dt = i % P, [torch.float32, torch.int64, torch.float64][i % 3]
            t = (torch.arange(5000 + 997 * i) + 100 * r).to(dt)
            hs.append(broadcast_async(t, f'hb{i:02d}', root, comm))
            want.append((torch.arange(5000 + 997 * i) + 100 * root).to(dt))
        for hd, w in zip(hs, want):
            got = hd.wait(timeout=120)
            assert not got.is_cuda and torch.equal(got, w)
        hs, want = [], []
        for i in range(4):
            dt = [torch.float32, torch.int32][i % 2]
            t = (torch.arange((r + 1 + i) * 3).reshape(-1, 3) + 1000 * r).to(dt)
            hs.append(allgather_async(t, f'hag{i}', comm))
            want.append(torch.cat([(torch.arange((q + 1 + i) * 3).reshape(-1, 3) + 1000 * q).to(dt) for q in range(P)]))
        for hd, w in zip(hs, want):
            got = hd.wait(timeout=120)
            assert not got.is_cuda and torch.equal(got, w)


def check_dp_training_cpu_model(ctx):
    """The DP wrapper on a CPU model (the reference's deployment: Keras on CPU tensors): initial
    weights broadcast, every gradient a keyed host allreduce, replicas equal one full-batch fp64
    step on the concatenated data."""
    torch, comm, P, r = ctx['torch'], ctx['comm'], ctx['P'], ctx['rank']
    from ddl.torch.parallelism.data import InitialParametersBroadcast, data_parallelism_distributed_optimizer_wrapper

    def model_fn(seed):
        torch.manual_seed(seed)
        return torch.nn.Sequential(torch.nn.Linear(16, 32), torch.nn.Tanh(), torch.nn.Linear(32, 4)).double()
    model = model_fn(99 + r)
    InitialParametersBroadcast(model, 0, communicator=comm).broadcast()
    ref = model_fn(99)
    for p, q in zip(model.parameters(), ref.parameters()):
        assert not p.is_cuda and torch.equal(p, q)
    opt = data_parallelism_distributed_optimizer_wrapper(torch.optim.SGD(model.parameters(), lr=0.1), comm)
    ref_opt = torch.optim.SGD(ref.parameters(), lr=0.1)
    g = torch.Generator().manual_seed(78)
    lib = ctx['lib']
    for step in range(3):
        xb = [torch.randn(8, 16, generator=g, dtype=torch.float64) for _ in range(P)]
        yb = [torch.randn(8, 4, generator=g, dtype=torch.float64) for _ in range(P)]
        opt.zero_grad()
        if step > 0:  # the gradients moved to pinned memory at step 0 survive zero_grad
            assert all(p.grad is not None and p.grad.is_pinned() and not p.grad.any() for p in model.parameters())
        torch.nn.functional.mse_loss(model(xb[r]), yb[r]).backward()
        plans0 = lib.ddl_get_config(b'host_zero_copy_plans')
        opt.step()
        if step > 0:  # one fp64 plan, unpacked by the kernel into the pinned gradients
            assert lib.ddl_get_config(b'host_zero_copy_plans') - plans0 == 1
        ref_opt.zero_grad()
        sum(torch.nn.functional.mse_loss(ref(xb[q]), yb[q]) for q in range(P)).div(P).backward()
        ref_opt.step()
    for p, q in zip(model.parameters(), ref.parameters()):
        assert torch.allclose(p, q, rtol=1e-12, atol=1e-12)


def check_dp_training_overlap(ctx):
    """overlap_backward: every gradient's keyed allreduce is submitted from its backward hook
    while autograd still runs; step() waits. Three steps equal one full-batch fp64 step each;
    then gradient accumulation — the first micro-batch's backward inside no_sync(), the second
    outside — equals the full-batch step over both micro-batches. GPU and CPU (pinned) models."""
    torch, comm, P, r = ctx['torch'], ctx['comm'], ctx['P'], ctx['rank']
    from ddl.torch.parallelism.data import InitialParametersBroadcast, data_parallelism_distributed_optimizer_wrapper
    for dev in ('cuda', 'cpu'):
        def model_fn(seed):
            torch.manual_seed(seed)
            return torch.nn.Sequential(torch.nn.Linear(16, 32), torch.nn.Tanh(), torch.nn.Linear(32, 32), torch.nn.Tanh(),
                                       torch.nn.Linear(32, 4)).double().to(dev)
        model = model_fn(555 + r)
        InitialParametersBroadcast(model, 0, communicator=comm).broadcast()
        ref = model_fn(555)
        opt = data_parallelism_distributed_optimizer_wrapper(torch.optim.SGD(model.parameters(), lr=0.05), comm,
                                                             overlap_backward=True)
        ref_opt = torch.optim.SGD(ref.parameters(), lr=0.05)
        g = torch.Generator().manual_seed(91)
        for step in range(4):
            micro = 2 if step == 3 else 1
            xb = [[torch.randn(8, 16, generator=g, dtype=torch.float64) for _ in range(P)] for _ in range(micro)]
            yb = [[torch.randn(8, 4, generator=g, dtype=torch.float64) for _ in range(P)] for _ in range(micro)]
            opt.zero_grad()
            for m in range(micro):
                ctxm = opt.no_sync() if m + 1 < micro else contextlib.nullcontext()
                with ctxm:
                    torch.nn.functional.mse_loss(model(xb[m][r].to(dev)), yb[m][r].to(dev)).backward()
            assert len(opt._grad_handles) == len(list(model.parameters()))  # all submitted by the hooks
            opt.step()
            ref_opt.zero_grad()
            for m in range(micro):
                sum(torch.nn.functional.mse_loss(ref(xb[m][q].to(dev)), yb[m][q].to(dev)) for q in range(P)).div(P).backward()
            ref_opt.step()
        for p, q in zip(model.parameters(), ref.parameters()):
            assert torch.allclose(p, q, rtol=1e-12, atol=1e-12), dev


def check_keyed_broadcast_allgather(ctx):
    """Keyed broadcasts with mixed roots and dtypes, keyed allgathers with per-rank first dims."""
    torch, comm, P, r = ctx['torch'], ctx['comm'], ctx['P'], ctx['rank']
    from ddl.torch.tensor_communicate import allgather_async, broadcast_async
    hs, want = [], []
    for i in range(12):
        root, dt = i % P, [torch.float32, torch.int64, torch.float16][i % 3]
        t = (torch.arange(1000 + 37 * i) + 100 * r).to(dt).cuda()
        hs.append(broadcast_async(t, f'b{i:02d}', root, comm))
        want.append((torch.arange(1000 + 37 * i) + 100 * root).to(dt))
    for hd, w in zip(hs, want):
        assert torch.equal(hd.wait(timeout=120).cpu(), w)
    hs, want = [], []
    for i in range(6):
        dt = [torch.float32, torch.int32][i % 2]
        t = (torch.arange((r + 1 + i) * 5).reshape(-1, 5) + 1000 * r).to(dt).cuda()
        hs.append(allgather_async(t, f'ag{i}', comm))
        want.append(torch.cat([(torch.arange((q + 1 + i) * 5).reshape(-1, 5) + 1000 * q).to(dt) for q in range(P)]))
    for hd, w in zip(hs, want):
        assert torch.equal(hd.wait(timeout=120).cpu(), w)


def check_host_resident(ctx):
    """allreduce of a CPU tensor: the chunked H2D -> ring -> D2H pipeline (4 slots), many chunks."""
    import _helpers as h
    torch, lib, comm, P, r = ctx['torch'], ctx['lib'], ctx['comm'], ctx['P'], ctx['rank']
    from ddl.torch.tensor_communicate import allreduce
    n = 1_000_003
    base = torch.randint(-1000, 1000, (n,), generator=torch.Generator().manual_seed(9))
    with h.config(lib, host_chunk_bytes=256 << 10):
        got = allreduce((base + r).to(torch.float32), comm)
    assert not got.is_cuda
    assert torch.equal(got, (base * P + P * (P - 1) // 2).to(torch.float32))


def check_dp_training(ctx):
    """Scripts-level drop-in: InitialParametersBroadcast, the DP optimizer wrapper (dense grads
    through keyed fused allreduces, a sparse embedding grad through allgather), MetricAverage.
    Replicas stay identical and equal one full-batch step on the concatenated data."""
    torch, comm, P, r, dist = ctx['torch'], ctx['comm'], ctx['P'], ctx['rank'], ctx['dist']
    from ddl.torch.parallelism.data import (InitialParametersBroadcast, MetricAverage,
                                            data_parallelism_distributed_optimizer_wrapper)

    def model_fn(seed):
        torch.manual_seed(seed)
        return torch.nn.Sequential(torch.nn.Linear(16, 32), torch.nn.Tanh(), torch.nn.Linear(32, 4)).double().cuda()
    model = model_fn(1234 + r)  # different initial weights on every rank
    InitialParametersBroadcast(model, 0, communicator=comm).broadcast()
    ref = model_fn(1234)  # rank 0's initial weights
    for p, q in zip(model.parameters(), ref.parameters()):
        assert torch.equal(p, q)
    opt = data_parallelism_distributed_optimizer_wrapper(torch.optim.SGD(model.parameters(), lr=0.1), comm)
    ref_opt = torch.optim.SGD(ref.parameters(), lr=0.1)
    g = torch.Generator().manual_seed(77)
    for step in range(3):
        xb = [torch.randn(8, 16, generator=g, dtype=torch.float64) for _ in range(P)]
        yb = [torch.randn(8, 4, generator=g, dtype=torch.float64) for _ in range(P)]
        opt.zero_grad()
        torch.nn.functional.mse_loss(model(xb[r].cuda()), yb[r].cuda()).backward()
        opt.step()
        ref_opt.zero_grad()  # mean of the per-rank losses = what the averaged gradients descend
        sum(torch.nn.functional.mse_loss(ref(xb[q].cuda()), yb[q].cuda()) for q in range(P)).div(P).backward()
        ref_opt.step()
    for p, q in zip(model.parameters(), ref.parameters()):
        assert torch.allclose(p, q, rtol=1e-12, atol=1e-12)
    # sparse gradient (IndexedSlices branch, tensor_communicate.py:26-30) through the wrapper
    emb = torch.nn.Embedding(10, 3, sparse=True).double().cuda()
    InitialParametersBroadcast(emb, 0, communicator=comm).broadcast()
    w0 = emb.weight.detach().clone()
    eopt = data_parallelism_distributed_optimizer_wrapper(torch.optim.SGD(emb.parameters(), lr=1.0), comm)
    eopt.zero_grad()
    emb(torch.tensor([r, r + 1], device='cuda')).sum().backward()
    eopt.step()
    want = w0.clone()
    for q in range(P):
        want[q] -= 1.0 / P
        want[q + 1] -= 1.0 / P
    assert torch.allclose(emb.weight.detach(), want)
    logs = MetricAverage(comm).on_epoch_end(0, {'loss': float(r), 'acc': 2.0 * r})
    assert logs == {'loss': (P - 1) / 2, 'acc': float(P - 1)}
    # the reference's DP script (examples/data_parallelism.py:73-101): lr scaled by the size, the
    # warm-up callback beside MetricAverage, the wrapped optimizer stepping under it
    from ddl.torch.parallelism.data import LearningRateWarmup
    base_lr, steps, warm = 0.05, 2, 2
    wopt = data_parallelism_distributed_optimizer_wrapper(
        torch.optim.SGD(model.parameters(), lr=base_lr * P, momentum=0.5), comm)
    cbs = [LearningRateWarmup(wopt, warmup_epochs=warm, steps_per_epoch=steps, communicator=comm),
           MetricAverage(comm)]
    cbs[0].on_train_begin()
    for e in range(warm + 1):
        cbs[0].on_epoch_begin(e)
        for b in range(steps):
            cbs[0].on_batch_begin(b)
            if e < warm:
                want = base_lr * P / P * ((e + (b + 1) / steps) * (P - 1) / warm + 1)
                assert abs(wopt.param_groups[0]['lr'] - want) < 1e-12, (e, b, wopt.param_groups[0]['lr'], want)
            wopt.zero_grad()
            torch.nn.functional.mse_loss(model(xb[r].cuda()), yb[r].cuda()).backward()
            wopt.step()
            cbs[0].on_batch_end(b)
            assert wopt.param_groups[0]['momentum'] == 0.5
        logs = cbs[1].on_epoch_end(e, cbs[0].on_epoch_end(e, {'loss': float(r)}))
        assert logs['loss'] == (P - 1) / 2 and abs(logs['lr'] - base_lr * P) < 1e-12 or e < warm - 1
    everyone = [None] * P
    dist.all_gather_object(everyone, [p.detach().cpu() for p in model.parameters()])
    for other in everyone[1:]:  # replicas stay identical under the schedule
        for a, b in zip(everyone[0], other):
            assert torch.equal(a, b)


def check_config_mismatch(ctx):
    """VERDICT r2 next #4(b) on the real engine: every rank changes a shared tunable at the same
    point, the last rank to a different value than the others — the next ddl_allreduce returns
    DDL_STATUS_CONFIG_MISMATCH on EVERY rank (the agreement runs before any program is built), a
    keyed request completes with that status on every rank (its round's tokens carry the hash),
    and once the values agree again both work."""
    import threading

    import _helpers as h
    from ddl.torch.cpp_backend import DONE_FN
    torch, lib, comm, P, r = ctx['torch'], ctx['lib'], ctx['comm'], ctx['P'], ctx['rank']
    s = torch.cuda.current_stream().cuda_stream
    x = torch.full((4099,), float(r), device='cuda')
    slice_bytes = (96 << 10) if r == P - 1 else (64 << 10)
    with h.config(lib, slice_bytes=slice_bytes):
        st = lib.ddl_allreduce(comm.id, x.data_ptr(), x.data_ptr(), x.numel(), h.DT_FLOAT, 0, s)
        assert st == 8, (st, lib.ddl_last_error())
        assert b'slice_bytes' in lib.ddl_last_error()
        got, ev = [], threading.Event()

        @DONE_FN
        def done(status, user):
            got.append(status)
            ev.set()
        y = torch.full((300,), float(r), device='cuda')
        assert lib.ddl_allreduce_submit(comm.id, b'cfg_mismatch', y.data_ptr(), y.data_ptr(), 300, h.DT_FLOAT, 0, s,
                                        done, None) == 0
        assert ev.wait(60) and got == [8], got
        assert lib.ddl_wait_all(comm.id) == 0
    # agreed again (every rank back to the same values): both paths work
    assert lib.ddl_allreduce(comm.id, x.data_ptr(), x.data_ptr(), x.numel(), h.DT_FLOAT, 0, s) == 0, lib.ddl_last_error()
    assert torch.equal(x, torch.full_like(x, float(P * (P - 1) // 2)))
    from ddl.torch.tensor_communicate import allreduce_async
    z = torch.full((300,), float(r), device='cuda')
    assert torch.equal(allreduce_async(z, 'cfg_ok', comm).wait(timeout=60), torch.full_like(z, float(P * (P - 1) // 2)))


def check_keyed_round_order(ctx):
    """keyed rounds (on the handler's private communicator) and direct
    ddl_allreduce calls (on the world) issued concurrently from two threads, with per-rank random
    pacing: every rank places every round after the same number of direct collectives (identical
    round logs), and every result is exact."""
    import random
    import threading
    import time

    import _helpers as h
    torch, lib, comm, P, r, dist = ctx['torch'], ctx['lib'], ctx['comm'], ctx['P'], ctx['rank'], ctx['dist']
    from ddl.torch.tensor_communicate import allreduce_async
    n_keyed, n_user = 24, 24
    rnd = random.Random(1000 + r)
    keyed = [torch.full((1000 + i,), float(r + i), device='cuda') for i in range(n_keyed)]
    errs = []

    def submitter():
        try:
            hs = []
            for i, t in enumerate(keyed):
                time.sleep(rnd.random() * 0.004)
                hs.append(allreduce_async(t, f'order_{i:02d}', comm))
            for i, hd in enumerate(hs):
                want = float(P * (P - 1) // 2 + P * i)
                assert torch.equal(hd.wait(timeout=120), torch.full_like(keyed[i], want)), i
        except Exception as e:  # noqa: BLE001
            errs.append(repr(e))
    th = threading.Thread(target=submitter)
    th.start()
    stream = torch.cuda.Stream()
    with torch.cuda.stream(stream):
        for j in range(n_user):
            time.sleep(rnd.random() * 0.004)
            u = torch.full((4099,), float(r * j), device='cuda')
            assert lib.ddl_allreduce(comm.id, u.data_ptr(), u.data_ptr(), u.numel(), h.DT_FLOAT, 0,
                                     stream.cuda_stream) == 0, lib.ddl_last_error()
            assert torch.equal(u, torch.full_like(u, float(j * P * (P - 1) // 2))), j
    th.join(timeout=180)
    assert not th.is_alive() and not errs, errs
    users, cnt = ctypes.c_longlong(), ctypes.c_int()
    rel = (ctypes.c_longlong * 4096)()
    assert lib.ddl_testing_round_log(comm.id, ctypes.byref(users), rel, 4096, ctypes.byref(cnt)) == 0
    mine = (users.value, list(rel[:min(cnt.value, 4096)]))
    everyone = [None] * P
    dist.all_gather_object(everyone, mine)
    assert all(e == mine for e in everyone), everyone
    assert mine[1] and mine[1] == sorted(mine[1]), mine


def check_control_link_lost(ctx):
    """a member's control link is lost right after it froze its user
    collectives for a keyed round (ddl_testing_control_fault on rank 1). Every rank's handler
    stops: the pending keyed request completes with an error on every rank, ddl_wait_all returns,
    and a later direct ddl_allreduce on the communicator returns the error instead of blocking
    behind the round that can no longer be placed. Run on its own (it leaves the handler dead)."""
    import threading

    import _helpers as h
    from ddl.torch.cpp_backend import DONE_FN
    from ddl.torch.tensor_communicate import allreduce_async
    torch, lib, comm, P, r = ctx['torch'], ctx['lib'], ctx['comm'], ctx['P'], ctx['rank']
    s = torch.cuda.current_stream().cuda_stream
    w = torch.full((500,), float(r), device='cuda')  # a healthy round first: the ring is up
    assert torch.equal(allreduce_async(w, 'warm', comm).wait(timeout=60), torch.full_like(w, float(P * (P - 1) // 2)))
    if r == 1:
        assert lib.ddl_testing_control_fault(1) == 0
    ctx['dist'].barrier()
    got, ev = [], threading.Event()

    @DONE_FN
    def done(status, user):
        got.append(status)
        ev.set()
    y = torch.full((300,), float(r), device='cuda')
    assert lib.ddl_allreduce_submit(comm.id, b'lost', y.data_ptr(), y.data_ptr(), 300, h.DT_FLOAT, 0, s,
                                    done, None) == 0, lib.ddl_last_error()
    assert ev.wait(60) and got and got[0] != 0, got
    lib.ddl_wait_all(comm.id)  # returns: it must not block on the stopped handler
    x = torch.full((4099,), float(r), device='cuda')
    st = lib.ddl_allreduce(comm.id, x.data_ptr(), x.data_ptr(), x.numel(), h.DT_FLOAT, 0, s)
    msg = lib.ddl_last_error().decode()
    assert st != 0 and 'handler stopped' in msg, (st, msg)


def check_resources(ctx):
    """Diagnostic for soak runs (tools/soak_mp.py): this rank's threads and open fds on stderr, so
    a leak across repeated checks shows as growth."""
    r = ctx['rank']
    threads = len(os.listdir('/proc/self/task'))
    fds = len(os.listdir('/proc/self/fd'))
    sys.stderr.write(f'[rank {r}] threads {threads} fds {fds}\n')
    sys.stderr.flush()


def check_graph_capture(ctx):
    """The data plane captured into a hipGraph and replayed over real multi-rank RCCL (the test
    transport synchronises the host and refuses capture): per capture mode (0 serial, 2 single-stream
    DAG) and schedule (direct, one-shot, gather-fold), K allreduces of different sizes captured once,
    then replayed three times on fresh inputs written into the captured buffers — every replay
    bit-exact vs MPICH's order on every rank."""
    import _helpers as h
    torch, lib, comm, P, r, ora = ctx['torch'], ctx['lib'], ctx['comm'], ctx['P'], ctx['rank'], ctx['oracle']
    sizes = (1000, 70_001, 300_001)
    for mode in (0, 2):
        for algo in (1, 2, 3):
            with h.config(lib, tune=0, algo=algo, reference_order=1, capture_mode=mode, slice_bytes=64 << 10):
                bufs = [(torch.empty(n, device='cuda'), torch.empty(n, device='cuda')) for n in sizes]
                gs = torch.cuda.Stream()
                with torch.cuda.stream(gs):  # warm-up outside the capture (staging, events)
                    for a, b in bufs:
                        a.fill_(1.0)
                        assert lib.ddl_allreduce(comm.id, a.data_ptr(), b.data_ptr(), a.numel(), h.DT_FLOAT, 0,
                                                 gs.cuda_stream) == 0, lib.ddl_last_error()
                torch.cuda.synchronize()
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g, stream=gs):
                    for a, b in bufs:
                        assert lib.ddl_allreduce(comm.id, a.data_ptr(), b.data_ptr(), a.numel(), h.DT_FLOAT, 0,
                                                 gs.cuda_stream) == 0, lib.ddl_last_error()
                for rep in range(3):
                    wants = []
                    for i, (a, b) in enumerate(bufs):
                        xs = [h.random_input(h.DT_FLOAT, a.numel(), 1000 * rep + 100 * i + 10 * algo + mode + q)
                              for q in range(P)]
                        a.copy_(torch.from_numpy(xs[r]))
                        b.fill_(float('nan'))
                        wants.append(ora.fold_ref_order(h.DT_FLOAT, xs))
                    torch.cuda.synchronize()
                    with torch.cuda.stream(gs):
                        g.replay()
                    torch.cuda.synchronize()
                    for (a, b), want in zip(bufs, wants):
                        assert b.cpu().numpy().tobytes() == want.tobytes(), (mode, algo, rep, a.numel())
                del g


def check_fullsize_mpich_hash(ctx):
    """Full-size parity over the real transport: every rank regenerates its
    64 Mi fp32 input of the golden case at this P (tests/golden/golden_fullsize.json: C3 at P = 8,
    and P = 5 / 7), runs the default schedule (tuner off) and its output must hash to MPICH 3.3.2's."""
    import _helpers as h
    torch, lib, comm, P, r = ctx['torch'], ctx['lib'], ctx['comm'], ctx['P'], ctx['rank']
    case = [c for c in h.fullsize_cases() if c[1] == P]
    assert case, f'no full-size golden case at P = {P}'
    name, _, n, digest, samples = case[0]
    x = np.random.default_rng(1234 + 7919 * r).standard_normal(n).astype(np.float32)
    a = torch.from_numpy(x).cuda()
    del x
    b = torch.full_like(a, float('nan'))
    with h.config(lib, tune=0, reference_order=1):
        st = lib.ddl_allreduce(comm.id, a.data_ptr(), b.data_ptr(), n, h.DT_FLOAT, 0,
                               torch.cuda.current_stream().cuda_stream)
        assert st == 0, lib.ddl_last_error()
        torch.cuda.synchronize()
    y = b.cpu().numpy()
    assert all(float(y[i]) == v for i, v in samples.items()), name
    assert h.sha256(y) == digest, name


FAULT_CHECKS = {'check_control_link_lost': check_control_link_lost, 'check_resources': check_resources,
                'check_fullsize_mpich_hash': check_fullsize_mpich_hash, 'check_graph_capture': check_graph_capture}


CHECKS = [check_reference_known_answers, check_schedules_vs_oracle, check_allreduce_batch, check_tuned_exact,
          check_keyed_fusion,
          check_keyed_reference_order, check_split_communicators_keyed, check_queue_classes, check_rccl_channel_bounds,
          check_keyed_host_requests,
          check_keyed_broadcast_allgather, check_host_resident, check_dp_training, check_dp_training_cpu_model,
          check_dp_training_overlap, check_config_mismatch, check_keyed_round_order]


def rccl_sockets_env(rank, world):
    """Environment that lets P processes on ONE GPU form a real multi-rank RCCL communicator:
    RCCL refuses two ranks of a communicator on one device only when it sees them on the same host
    (same host hash and bus id, "Duplicate GPU detected"). NCCL_HOSTID gives every rank a host of
    its own, so RCCL connects them through its network transport — sockets on the loopback
    interface — instead of xGMI. Everything above the wire is the production path: ddl_init's
    ncclCommInitRankConfig at size P, ncclCommSplit across ranks, RcclTransport's send / recv
    pairs between processes, ncclAllGather, the tuner's ncclAllReduce(MAX). Test infrastructure
    only (the rates are a socket's, not xGMI's)."""
    env = {'NCCL_HOSTID': f'ddl-test-host-{rank}-of-{world}', 'NCCL_SOCKET_IFNAME': 'lo', 'NCCL_IB_DISABLE': '1'}
    if os.environ.get('DDL_MP_HW_QUEUES'):  # hardware queues per rank process (HIP reads it at init)
        env['GPU_MAX_HW_QUEUES'] = os.environ['DDL_MP_HW_QUEUES']
    return env


def worker(rank, world, port, q, only=None, transport='gloo'):
    results = []
    try:
        if transport == 'rccl':  # before anything initialises RCCL in this process
            os.environ.update(rccl_sockets_env(rank, world))
        for p in (os.path.join(ROOT, 'experiment-distributed-deep-learning_amd'), HERE, os.path.join(ROOT, 'tools')):
            if p not in sys.path:
                sys.path.insert(0, p)
        os.environ['MASTER_ADDR'] = '127.0.0.1'
        os.environ['MASTER_PORT'] = str(port)
        import datetime

        import torch
        import torch.distributed as dist
        dist.init_process_group('gloo', rank=rank, world_size=world, timeout=datetime.timedelta(seconds=90))
        torch.cuda.set_device(0)
        import _helpers as h
        from ddl.torch.communicator import Communicator
        from ddl.torch.cpp_backend import CPPBackend, check
        lib = CPPBackend.c_api()
        import gloo_transport
        # engine placement knobs for A/B runs (read when the executors / handlers are created)
        for env, key in (('DDL_MP_NUMA_BIND', b'host_numa_bind'), ('DDL_MP_CU_MASK', b'compute_cu_mask'),
                         ('DDL_MP_QUEUE_ISOLATION', b'queue_isolation')):
            if os.environ.get(env):
                check(lib.ddl_set_config(key, int(os.environ[env])), 'ddl_set_config')
        if transport == 'rccl':
            from ddl.torch.communicator import init
            init(rank, world, 0)  # the product's bootstrap: ddl_init over a real RCCL communicator
            cbs = None
        else:
            cbs = gloo_transport.init_world(lib, dist, torch, rank, world)  # noqa: F841 (keep alive)
        comm = Communicator.world()
        assert comm.size == world and comm.rank == rank
        kind, tranks = ctypes.c_int(), ctypes.c_int()
        check(lib.ddl_comm_transport(comm.id, ctypes.byref(kind), ctypes.byref(tranks)), 'ddl_comm_transport')
        assert (kind.value, tranks.value) == ((1, world) if transport == 'rccl' else (2, world)), (kind, tranks)
        # the configured schedule unless a check turns the tuner on (check_tuned_exact): tuning
        # every new size class through gloo host copies is what makes these runs slow at P = 8
        check(lib.ddl_set_config(b'tune', 0), 'ddl_set_config')
        # keyed rounds waited for one by one (the reference's behaviour) when the test asks
        check(lib.ddl_set_config(b'pipeline_rounds', int(os.environ.get('DDL_MP_PIPELINE_ROUNDS', 1))),
              'ddl_set_config')
        ctx = {'torch': torch, 'dist': dist, 'lib': lib, 'comm': comm, 'P': world, 'rank': rank,
               'oracle': h.Oracle(), 'transport': transport,
               'queue_isolation': lib.ddl_get_config(b'queue_isolation')}
        import time
        if os.environ.get('DDL_MP_STACKS_S'):  # soak diagnostics: Python stacks of a hung rank
            import faulthandler
            faulthandler.dump_traceback_later(float(os.environ['DDL_MP_STACKS_S']), repeat=True)
        by_name = {**{f.__name__: f for f in CHECKS}, **FAULT_CHECKS}  # `only`: any checks by name, in order
        for fn in ([by_name[n] for n in only] if only else CHECKS):
            try:
                t0 = time.perf_counter()
                fn(ctx)
                results.append((fn.__name__, True, ''))
                if rank == 0:
                    line = f'[P={world} {transport}] {fn.__name__}: {time.perf_counter() - t0:.1f} s\n'
                    sys.stderr.write(line)
                    sys.stderr.flush()
                    if os.environ.get('DDL_MP_PROGRESS_FILE'):  # long GPU runs: progress outside pytest's capture
                        with open(os.environ['DDL_MP_PROGRESS_FILE'], 'a') as f:
                            f.write(line)
            except Exception:
                results.append((fn.__name__, False, traceback.format_exc()[-1500:]))
                break  # a failed collective leaves the ranks out of step: stop here
        dist.barrier()
        from ddl.torch.communicator import finalize
        finalize()
    except Exception:
        results.append(('setup', False, traceback.format_exc()[-2000:]))
    q.put((rank, results))
