"""Completion groups (ddl_completion_*, csrc/completion.cpp): the native done callback the torch
mirror hands the engine for keyed requests, so completing a request costs no Python callback
(a Python done() per tensor cost 40-60 ms per 4096-tensor batch). CPU only: the engine's
completion thread is stood in for by threads calling ddl_completion_done, as the engine does
(include/ddl_amd.h: done(status, user) with user = the slot's pointer)."""
import ctypes
import threading
import time

import pytest


def _slots(lib, g, n):
    arr = (ctypes.c_void_p * n)()
    assert lib.ddl_completion_slots(g, 0, n, arr) == 0
    return list(arr)


def test_slots_complete_once_and_wait_returns_status(lib):
    g = lib.ddl_completion_create(3)
    assert g
    s = _slots(lib, g, 3)
    try:
        assert lib.ddl_completion_poll(g, None, 0) == 3
        st = ctypes.c_int(-5)
        assert lib.ddl_completion_wait(g, 1, 0.0, ctypes.byref(st)) == 2  # a test: pending
        t0 = time.perf_counter()
        assert lib.ddl_completion_wait(g, 1, 0.05, ctypes.byref(st)) == 2  # still pending after 50 ms
        assert time.perf_counter() - t0 >= 0.04
        lib.ddl_completion_done(7, s[1])
        lib.ddl_completion_done(0, s[1])  # a slot completes once
        assert lib.ddl_completion_wait(g, 1, -1.0, ctypes.byref(st)) == 0 and st.value == 7
        arr = (ctypes.c_int * 3)()
        assert lib.ddl_completion_poll(g, arr, 3) == 2 and list(arr) == [-1, 7, -1]
        bad = (ctypes.c_void_p * 1)()
        assert lib.ddl_completion_slots(g, 2, 2, bad) == 3 and lib.ddl_completion_wait(g, 3, 0.0, None) == 3
    finally:
        for i in (0, 2):  # complete the rest, then let go: the group is freed
            lib.ddl_completion_done(0, s[i])
        lib.ddl_completion_destroy(g)


def test_waiter_wakes_when_another_thread_completes(lib):
    k = 4096
    g = lib.ddl_completion_create(k)
    slots = _slots(lib, g, k)

    def engine():  # completions in order, as the engine fires done() in plan order
        for i, s in enumerate(slots):
            lib.ddl_completion_done(0 if i % 97 else 3, s)
    t = threading.Thread(target=engine)
    t.start()
    st = ctypes.c_int()
    for i in range(k):
        assert lib.ddl_completion_wait(g, i, 30.0, ctypes.byref(st)) == 0
        assert st.value == (0 if i % 97 else 3)
    t.join()
    assert lib.ddl_completion_poll(g, None, 0) == 0
    lib.ddl_completion_destroy(g)


def test_owner_may_let_go_before_the_engine_completes(lib):
    """The binding drops its handles without waiting: the group lives until the last done()."""
    for _ in range(50):
        g = lib.ddl_completion_create(4)
        slots = _slots(lib, g, 4)
        lib.ddl_completion_done(0, slots[0])
        lib.ddl_completion_destroy(g)  # owner gone, 3 slots still pending: not freed yet
        th = [threading.Thread(target=lib.ddl_completion_done, args=(0, s)) for s in slots[1:]]
        for x in th:
            x.start()
        for x in th:
            x.join()  # the last done() freed it (ASAN: tools/asan_cpu_tests.sh)
    g = lib.ddl_completion_create(0)  # an empty group is freed at once by its owner
    assert lib.ddl_completion_poll(g, None, 0) == 0
    lib.ddl_completion_destroy(g)


def test_torch_mirror_handles_over_a_group(lib):
    """The mirror's _NativeHandle / _Completion: done() / wait() read the slot, a refused
    submission's slots are completed with its status, all statuses are cached once every slot
    completed, and the group keeps the tensors alive until then (swept at the next group's
    creation)."""
    import torch

    from ddl.torch import tensor_communicate as tc
    from ddl.torch.cpp_backend import DDLError
    a, b = torch.zeros(4), torch.ones(4)
    grp = tc._Completion(2, (a, b))
    hs = [tc._NativeHandle('a', a, (a,), grp, 0), tc._NativeHandle('b', b, (b,), grp, 1)]
    assert not hs[0].done()
    with pytest.raises(TimeoutError):
        hs[0].wait(timeout=0.01)
    assert grp in tc._Completion._inflight
    lib.ddl_completion_done(0, grp.slots()[0])
    assert hs[0].done() and hs[0].wait() is a and grp.final is None and grp.keep is not None
    grp.fail([1], 7)  # a refused submission: every slot complete, the tensors are let go
    assert grp.keep is None
    with pytest.raises(DDLError) as e:
        hs[1].wait(timeout=1)
    assert e.value.status == 7 and grp.final == [0, 7]
    tc._Completion(0, ())  # the next group sweeps the completed one
    assert grp not in tc._Completion._inflight
    one = tc._Completion(1, (a,))  # a single request: its wait() releases the tensors
    h = tc._NativeHandle('c', a, (a,), one, 0)
    lib.ddl_completion_done(0, one.slots()[0])
    assert h.wait() is a and one.keep is None and one.final == [0]


def test_completed_groups_behind_a_pending_one_are_released(lib):
    """groups complete out of submission order (keyed requests wait for every rank,
    communicators complete independently). A group left pending at the head must not pin the
    tensors of the completed groups behind it: once the deque doubled since the last full sweep,
    every completed group goes, and the deque stays bounded."""
    import torch

    from ddl.torch import tensor_communicate as tc
    stuck = tc._Completion(1, (torch.zeros(1),))  # never completed until the end
    done = []
    for i in range(300):
        g = tc._Completion(1, (torch.zeros(1),))
        lib.ddl_completion_done(0, g.slots()[0])
        done.append(g)
    assert stuck in tc._Completion._inflight
    assert len(tc._Completion._inflight) < 130, len(tc._Completion._inflight)
    assert sum(g.keep is not None for g in done) < 130
    lib.ddl_completion_done(0, stuck.slots()[0])
    tc._Completion(0, ())
    assert stuck not in tc._Completion._inflight and stuck.keep is None


def test_native_completion_is_cheaper_than_python_callbacks(lib):
    """4096 completions fired from a native thread (an ordinary ddl_done_fn caller), then waited
    for handle by handle through the mirror: the whole batch in a few ms (a Python done() per
    request costs ~10 us each)."""
    from ddl.torch import tensor_communicate as tc
    k = 4096
    best = float('inf')
    for _ in range(3):
        t0 = time.perf_counter()
        grp = tc._Completion(k, ())
        hs = [tc._NativeHandle(str(i), None, (), grp, i) for i in range(k)]
        slots = grp.slots()
        th = threading.Thread(target=lambda: [lib.ddl_completion_done(0, s) for s in slots])
        th.start()
        for h in hs:
            h.wait(timeout=30)
        th.join()
        best = min(best, time.perf_counter() - t0)
    assert best < 0.25, best  # generous: the CI container is shared
