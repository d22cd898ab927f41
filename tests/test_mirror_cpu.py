"""The torch mirror's keyed batch submission (ddl.torch.tensor_communicate.allreduce_async_batch)
on CPU: what it hands the C-ABI (ddl_allreduce_submit_batch_mem, include/ddl_amd.h) for a batch
of host tensors — keys, in / out pointers, element counts, dtypes and one completion slot per
request — in place (the DP wrapper's form), out of place and with outputs it allocates, and how a
refused submission completes its handles. The engine's side is stood in for by a recording
submit that completes the slots through the library's own ddl_completion_done, as the engine's
done() does; every other entry point is the real library's."""
import ctypes

import pytest
import torch


class _Recorder:
    def __init__(self, real, status=0):
        self._real, self.status, self.calls = real, status, []

    def __getattr__(self, name):
        return getattr(self._real, name)

    def ddl_get_config(self, key):
        return 0 if key == b'host_register_cache_bytes' else self._real.ddl_get_config(key)

    def ddl_allreduce_submit_batch_mem(self, comm, m, keys, ins, outs, ns, dts, op, mem, stream, done, users):
        self.calls.append({'comm': comm, 'm': m, 'keys': [keys[i] for i in range(m)],
                           'ins': [ins[i] for i in range(m)], 'outs': [outs[i] for i in range(m)],
                           'same_array': ins is outs, 'ns': [ns[i] for i in range(m)],
                           'dts': [dts[i] for i in range(m)], 'op': op, 'mem': mem, 'stream': stream,
                           'done': ctypes.cast(done, ctypes.c_void_p).value,
                           'users': [users[i] for i in range(m)]})
        if self.status == 0:
            for i in range(m):
                self._real.ddl_completion_done(0, users[i])
        return self.status


class _Comm:
    id = 77


@pytest.fixture
def recorder(lib, monkeypatch):
    from ddl.torch.cpp_backend import CPPBackend
    rec = _Recorder(lib)
    monkeypatch.setattr(CPPBackend, 'c_api', staticmethod(lambda: rec))
    return rec


def _tensors():
    return [torch.arange(5, dtype=torch.float32), torch.ones(3, dtype=torch.float16),
            torch.zeros(0, dtype=torch.float64), torch.full((7,), 2, dtype=torch.int32)]


def test_in_place_batch_passes_one_pointer_array(recorder, lib):
    from ddl.torch import cpp_backend as cb
    from ddl.torch.tensor_communicate import allreduce_async_batch
    ts = _tensors()
    names = ['b', 'a', 'c', 'd']
    hs = allreduce_async_batch(ts, names, _Comm(), outputs=ts)
    (c,) = recorder.calls
    assert c['comm'] == 77 and c['m'] == 4 and c['mem'] == cb.MEMORY_HOST and c['op'] == cb.OP_SUM
    assert c['keys'] == [n.encode() for n in names]
    assert c['ins'] == [t.data_ptr() or None for t in ts] and c['same_array']
    assert c['ns'] == [5, 3, 0, 7] and c['dts'] == [1, 19, 2, 3] and c['stream'] in (0, None)
    assert c['done'] == ctypes.cast(lib.ddl_completion_done, ctypes.c_void_p).value  # native done()
    assert len(set(c['users'])) == 4 and all(c['users'])
    for h, t in zip(hs, ts):
        assert h.done() and h.wait(timeout=5) is t


def test_out_of_place_and_allocated_outputs(recorder):
    from ddl.torch.tensor_communicate import allreduce_async_batch
    ts = _tensors()[:2]
    outs = [torch.empty_like(t) for t in ts]
    hs = allreduce_async_batch(ts, ['x', 'y'], _Comm(), outputs=outs)
    c = recorder.calls[-1]
    assert not c['same_array'] and c['ins'] == [t.data_ptr() for t in ts]
    assert c['outs'] == [o.data_ptr() for o in outs]
    assert [h.wait(timeout=5) for h in hs] == outs
    hs = allreduce_async_batch(ts, ['x', 'y'], _Comm())  # the mirror allocates the outputs
    c = recorder.calls[-1]
    got = [h.wait(timeout=5) for h in hs]
    assert c['outs'] == [g.data_ptr() for g in got] and all(g.data_ptr() != t.data_ptr() for g, t in zip(got, ts))
    assert all(g.shape == t.shape and g.dtype == t.dtype for g, t in zip(got, ts))


def test_refused_batch_completes_every_handle_with_its_status(recorder):
    from ddl.torch.cpp_backend import DDLError
    from ddl.torch.tensor_communicate import allreduce_async_batch
    recorder.status = 7  # DDL_STATUS_DUPLICATE_KEY
    with pytest.raises(DDLError) as e:
        allreduce_async_batch(_tensors(), ['k1', 'k2', 'k3', 'k4'], _Comm())
    assert e.value.status == 7 and len(recorder.calls) == 1


def test_batch_argument_checks(recorder):
    from ddl.torch.tensor_communicate import allreduce_async_batch
    ts = _tensors()
    with pytest.raises(ValueError):
        allreduce_async_batch(ts, ['only one'], _Comm())
    with pytest.raises(ValueError):  # a non-contiguous input
        allreduce_async_batch([torch.ones(4, 4).t()], ['t'], _Comm())
    with pytest.raises(TypeError):
        allreduce_async_batch([torch.ones(4, dtype=torch.int8)], ['i8'], _Comm())
    assert allreduce_async_batch([], [], _Comm()) == [] and not recorder.calls


def test_argument_errors_leave_no_pending_group(recorder):
    """A dtype or key the mirror rejects raises before any completion group exists: a group whose
    slots are never submitted would stay pending at the head of the in-flight queue and keep every
    later batch's tensors alive."""
    from ddl.torch import tensor_communicate as tc
    before = len(tc._Completion._inflight)
    for bad in ([torch.ones(4, dtype=torch.int8)], [torch.ones(4, dtype=torch.bool)]):
        with pytest.raises(TypeError):
            tc.allreduce_async_batch(bad, ['bad'], _Comm())
        with pytest.raises(TypeError):
            tc.allreduce_async(bad[0], 'bad', _Comm())
        with pytest.raises(TypeError):
            tc.broadcast_async(bad[0], 'bad', 0, _Comm())
    with pytest.raises(AttributeError):  # a key that is not a string
        tc.allreduce_async_batch([torch.ones(2)], [3], _Comm())
    assert len(tc._Completion._inflight) <= before
    assert not recorder.calls


def test_failed_submission_call_completes_the_slots(recorder):
    """An exception inside the submission call itself (here: the recording submit raising) fails
    the batch's slots, so the group cannot stay pending."""
    from ddl.torch import tensor_communicate as tc

    def boom(*a):
        raise RuntimeError('boom')
    recorder.ddl_allreduce_submit_batch_mem = boom
    ts = [torch.ones(3), torch.ones(2)]
    with pytest.raises(RuntimeError):
        tc.allreduce_async_batch(ts, ['p', 'q'], _Comm())
    grp = tc._Completion._inflight[-1]
    assert grp.keep is None and grp.count == 2  # every slot completed: the tensors are let go
    assert tc.CPPBackend.c_api().ddl_completion_poll(grp.ptr, None, 0) == 0
