"""Tensor collectives (mirror of reference src/py/ddl/tensorflow/tensor_communicate.py:9-129).

`allreduce(tensor, communicator)` returns a new tensor holding the elementwise SUM over the
communicator's ranks — as the reference's `Allreduce` op does (AllreduceOp.cc:32-66, output
allocated like the input). `allreduce_gradient` divides by the size. `allreduce_async` is the
keyed request path (the TF op's asynchronous `handleRequest`): requests registered under
a key are negotiated across ranks, fused by dtype in key order and completed through a
callback.

Device tensors stay in HBM; the call is ordered on torch's current stream and does not
synchronise the host. A host (CPU) tensor — the reference's deployment case — is staged
through pinned memory to the GPU, reduced there and copied back.
"""
import bisect
import collections
import ctypes
import itertools
import threading
import weakref

import torch

from ddl.torch import cpp_backend as cb
from ddl.torch.communicator import Communicator
from ddl.torch.cpp_backend import CPPBackend, check
from ddl.torch.util import (current_stream_handle, ddl_dtype, memory_kind, require_device_tensor,
                           stream_handle_for)


def _comm(communicator):
    return Communicator.world() if communicator is None else communicator


def _allreduce_device(src: torch.Tensor, dst: torch.Tensor, communicator: Communicator) -> None:
    require_device_tensor(src, 'allreduce input')
    require_device_tensor(dst, 'allreduce output')
    check(CPPBackend.c_api().ddl_allreduce(
        communicator.id, src.data_ptr(), dst.data_ptr(), src.numel(), ddl_dtype(src), cb.OP_SUM,
        current_stream_handle(src.device)), 'ddl_allreduce')


def allreduce(tensor: torch.Tensor, communicator: Communicator = None) -> torch.Tensor:
    """Sum `tensor` over all ranks of `communicator`; returns a new tensor."""
    communicator = _comm(communicator)
    if tensor.is_cuda:
        src = tensor.contiguous()
        out = torch.empty_like(src)
        _allreduce_device(src, out, communicator)
        return out.view_as(tensor)
    # host-resident bucket: the engine's chunked H2D -> device ring -> D2H pipeline
    src = tensor.contiguous()
    out = torch.empty(tensor.shape, dtype=tensor.dtype, pin_memory=True)
    check(CPPBackend.c_api().ddl_allreduce_host(
        communicator.id, src.data_ptr(), out.data_ptr(), src.numel(), ddl_dtype(src), cb.OP_SUM),
        'ddl_allreduce_host')
    return out


def allreduce_(tensor: torch.Tensor, communicator: Communicator = None) -> torch.Tensor:
    """In-place variant of `allreduce` (device tensors only)."""
    communicator = _comm(communicator)
    _allreduce_device(tensor, tensor, communicator)
    return tensor


def allreduce_batch_(tensors, communicator: Communicator = None):
    """In-place SUM of every device tensor in `tensors` (one dtype) over the ranks, as ONE grouped
    collective (ddl_allreduce_batch): a DDP-style bucket list reduced with one RCCL group per tick
    and the folds of up to 8 buckets per kernel launch. With reference_order 1 (the default) each
    result is bit for bit what `allreduce_` gives that tensor alone (MPICH's order for its own
    size); with reference_order 0 the batch schedule's order may differ from a solo call's in the
    last bits (include/ddl_amd.h). Every rank passes the same shapes in the same order."""
    communicator = _comm(communicator)
    tensors = list(tensors)
    if not tensors:
        return tensors
    dt = ddl_dtype(tensors[0])
    for t in tensors:
        require_device_tensor(t, 'allreduce_batch_ tensor')
        if ddl_dtype(t) != dt or not t.is_contiguous():
            raise ValueError('allreduce_batch_ needs contiguous tensors of one dtype')
    k = len(tensors)
    ptrs = (ctypes.c_void_p * k)(*[t.data_ptr() for t in tensors])
    counts = (ctypes.c_size_t * k)(*[t.numel() for t in tensors])
    check(CPPBackend.c_api().ddl_allreduce_batch(communicator.id, k, ptrs, ptrs, counts, dt, cb.OP_SUM,
                                                  current_stream_handle(tensors[0].device)), 'ddl_allreduce_batch')
    return tensors


def allreduce_gradient(tensor: torch.Tensor, communicator: Communicator = None,
                       return_mean: bool = True) -> torch.Tensor:
    """Dense gradient: allreduce, then divide by the size (tensor_communicate.py:21-25).

    Sparse gradient (torch sparse COO, the counterpart of TF's IndexedSlices, :26-30): the
    values and the indices are allgathered — every rank's rows in rank order — and the mean
    divides the values; duplicate indices stay uncoalesced, as IndexedSlices keeps them.
    """
    communicator = _comm(communicator)
    if tensor.is_sparse:
        values = allgather(tensor._values(), communicator)
        if return_mean:
            values = values / communicator.size
        indices = allgather(tensor._indices().t().contiguous(), communicator).t()
        return torch.sparse_coo_tensor(indices, values, tensor.shape)
    summed = allreduce(tensor, communicator)
    if return_mean:
        summed.div_(communicator.size)
    return summed


def broadcast(tensor: torch.Tensor, root_rank: int, communicator: Communicator = None) -> torch.Tensor:
    """Returns root's `tensor` on every rank (TF op Broadcast, tensor_communicate.py:58-68):
    a new tensor; `tensor` itself is left as it was."""
    communicator = _comm(communicator)
    if tensor.is_cuda:
        out = tensor.contiguous().clone()
        return broadcast_(out, root_rank, communicator)
    out = broadcast_(tensor.contiguous().to('cuda'), root_rank, communicator)
    return out.cpu()


def broadcast_(tensor: torch.Tensor, root_rank: int, communicator: Communicator = None) -> torch.Tensor:
    """In-place broadcast of a device tensor from `root_rank` (Communicator::broadcast)."""
    communicator = _comm(communicator)
    require_device_tensor(tensor, 'broadcast tensor')
    check(CPPBackend.c_api().ddl_broadcast(communicator.id, tensor.data_ptr(), tensor.numel(), ddl_dtype(tensor),
                                           int(root_rank), current_stream_handle(tensor.device)), 'ddl_broadcast')
    return tensor


def allgather(tensor: torch.Tensor, communicator: Communicator = None) -> torch.Tensor:
    """Concatenation along dim 0 of every rank's `tensor`, in rank order (TF op Allgather,
    tensor_communicate.py:45-55; first dims may differ per rank, the other dims may not —
    MPIRingTokenCommunication.cc:160-364). The first dims are exchanged first (one small
    allgather and a host read), then the data lands straight in the output."""
    import ctypes
    communicator = _comm(communicator)
    host = not tensor.is_cuda
    src = tensor.contiguous().to('cuda') if host else tensor.contiguous()
    if src.dim() == 0:
        src = src.reshape(1)
    P = communicator.size
    lib = CPPBackend.c_api()
    stream = current_stream_handle(src.device)
    dims = torch.empty(P, dtype=torch.int64, device=src.device)
    mine = torch.tensor([src.shape[0]], dtype=torch.int64, device=src.device)
    check(lib.ddl_allgather(communicator.id, mine.data_ptr(), 1, dims.data_ptr(), 1, cb.DT_INT64, stream),
          'ddl_allgather')
    first = [int(d) for d in dims.cpu().tolist()]
    row = 1
    for d in src.shape[1:]:
        row *= d
    out = torch.empty((sum(first),) + tuple(src.shape[1:]), dtype=src.dtype, device=src.device)
    counts = (ctypes.c_size_t * P)(*[f * row for f in first])
    displs = (ctypes.c_size_t * P)(*[sum(first[:q]) * row for q in range(P)])
    check(lib.ddl_allgatherv(communicator.id, src.data_ptr(), src.numel(), out.data_ptr(), counts, displs,
                             ddl_dtype(src), stream), 'ddl_allgatherv')
    return out.cpu() if host else out


# ---- keyed asynchronous requests -----------------------------------------------------------
class Handle:
    """Completion handle of a keyed request (the TF op's pending `done` callback)."""
    __slots__ = ('key', 'output', '_keep', '_event', 'status', '__dict__', '__weakref__')

    def __init__(self, key: str, output: torch.Tensor, keep_alive):
        self.key = key
        self.output = output
        self._keep = keep_alive
        self._event = threading.Event()
        self.status = None

    def done(self) -> bool:
        return self._event.is_set()

    def wait(self, timeout: float = None) -> torch.Tensor:
        if not self._event.wait(timeout):
            raise TimeoutError(f'request {self.key!r} did not complete')
        self._keep = None
        if self.status != cb.STATUS_OK:
            raise cb.DDLError(self.status, f'request {self.key!r}', '')
        return self.output


_pending_lock = threading.Lock()  # keyed allgathers in flight (_gathers)
_ids = itertools.count(1)


class _Completion:
    """A completion group of the engine (ddl_completion_*, csrc/completion.cpp): the engine's
    done() is native and stores each request's status in its slot, so completing a request costs
    no Python callback (~10 us of interpreter time each: 40-60 ms per 4096-tensor batch, DESIGN
    §7); a handle blocks in C++ with the GIL released, and once every slot has completed one poll
    caches all statuses, so the rest of a batch's waits are list reads. The group holds the
    requests' tensors until every slot has completed (swept at later submissions), so a handle
    dropped without wait() cannot free memory the engine still reads or writes; the engine frees
    the group once its owner let go AND every slot completed."""
    __slots__ = ('ptr', 'count', 'keep', 'final', '__weakref__')
    _inflight = collections.deque()  # groups in submission order, slots maybe pending: their tensors
    _inflight_lock = threading.Lock()
    _sweep_at = 64  # a full sweep of _inflight once it holds this many groups (then 2x the survivors)

    def __init__(self, count: int, keep):
        lib = CPPBackend.c_api()
        self.ptr = lib.ddl_completion_create(count)
        if not self.ptr:
            raise MemoryError('ddl_completion_create')
        self.count, self.keep, self.final = count, keep, None
        weakref.finalize(self, lib.ddl_completion_destroy, self.ptr)
        with _Completion._inflight_lock:
            # release the groups that completed. Most complete in submission order (one
            # communicator's rounds), so the head is swept at every submission; but keyed requests
            # complete only once every rank registered the key, and communicators complete
            # independently, so a pending group may sit in front of completed ones:
            # once the deque doubled since the last full sweep, every group is looked at. O(1)
            # amortised per submission either way.
            q = _Completion._inflight
            while q and (q[0].keep is None or lib.ddl_completion_poll(q[0].ptr, None, 0) == 0):
                q.popleft().keep = None
            if len(q) >= _Completion._sweep_at:
                live = collections.deque()
                for g in q:
                    if g.keep is None or lib.ddl_completion_poll(g.ptr, None, 0) == 0:
                        g.keep = None
                    else:
                        live.append(g)
                _Completion._inflight = q = live
                _Completion._sweep_at = max(64, 2 * len(live))
            q.append(self)

    def slots(self, first: int = 0, count: int = None):
        """The `user` pointers of slots [first, first + count) (a ctypes array)."""
        count = self.count - first if count is None else count
        arr = (ctypes.c_void_p * count)()
        check(CPPBackend.c_api().ddl_completion_slots(self.ptr, first, count, arr), 'ddl_completion_slots')
        return arr

    def status(self, index: int, timeout: float = None) -> int:
        """Slot `index`'s status once it completed (TimeoutError after `timeout` seconds)."""
        if self.final is not None:
            return self.final[index]
        lib = CPPBackend.c_api()
        st = ctypes.c_int()
        if lib.ddl_completion_wait(self.ptr, index, -1.0 if timeout is None else float(timeout),
                                   ctypes.byref(st)) != cb.STATUS_OK:
            raise TimeoutError('request did not complete')
        if lib.ddl_completion_poll(self.ptr, None, 0) == 0:
            # every slot completed: cache the statuses and let the tensors go (a host tensor's
            # storage finalizer may release its registration now, as with the reference's op,
            # whose inputs are released when its done() has run)
            arr = (ctypes.c_int * self.count)()
            lib.ddl_completion_poll(self.ptr, arr, self.count)
            self.final = list(arr)
            self.keep = None
        return st.value

    def fail(self, indices, status):
        """The submission was refused: nothing will complete these slots but us."""
        lib = CPPBackend.c_api()
        slots = self.slots()
        for i in indices:
            lib.ddl_completion_done(status, slots[i])
        if lib.ddl_completion_poll(self.ptr, None, 0) == 0:
            self.keep = None


_NATIVE_DONE = []
_STATUS_ERROR_UNKNOWN = 2  # include/ddl_amd.h DDL_STATUS_ERROR_UNKNOWN


def _native_done():
    """ddl_completion_done as a ddl_done_fn argument (the C function itself: no Python callback)."""
    if not _NATIVE_DONE:
        lib = CPPBackend.c_api()
        _NATIVE_DONE.append(cb.DONE_FN(ctypes.cast(lib.ddl_completion_done, ctypes.c_void_p).value))
    return _NATIVE_DONE[0]


class _NativeHandle(Handle):
    """Handle of a request completed through a completion group (no Python done callback)."""
    __slots__ = ('_group', '_index')

    def __init__(self, key: str, output: torch.Tensor, keep_alive, group: _Completion, index: int):
        # (no threading.Event: the slot is the completion)
        self.key, self.output, self._keep, self.status = key, output, keep_alive, None
        self._group, self._index = group, index

    def done(self) -> bool:
        try:
            self.status = self._group.status(self._index, 0.0)
        except TimeoutError:
            return False
        return True

    def wait(self, timeout: float = None) -> torch.Tensor:
        try:
            self.status = self._group.status(self._index, timeout)
        except TimeoutError:
            raise TimeoutError(f'request {self.key!r} did not complete') from None
        self._keep = None
        if self.status != cb.STATUS_OK:
            raise cb.DDLError(self.status, f'request {self.key!r}', '')
        return self.output


# Host ranges the engine's registration cache may hold, as the torch mirror submitted them (see
# _watch_host): start address -> (end, id of the storage object, its finalizer); _watched_starts
# keeps the starts sorted for the overlap lookup.
_watched = {}
_watched_starts = []
_watched_by_storage = {}  # id of the storage object -> the start it was recorded at
_watched_lock = threading.Lock()


def _release_range(lo, hi):
    try:
        CPPBackend.c_api().ddl_host_unregister(lo, hi - lo)
    except Exception:  # noqa: BLE001 (interpreter shutdown: the library may be gone)
        pass


def _forget_locked(lo):
    entry = _watched.pop(lo, None)
    if entry is not None:
        _watched_starts.pop(bisect.bisect_left(_watched_starts, lo))
        if _watched_by_storage.get(entry[1]) == lo:
            del _watched_by_storage[entry[1]]
    return entry


def _on_storage_freed(lo, key):
    """Finalizer of a watched storage: its memory is about to be released."""
    with _watched_lock:
        entry = _watched.get(lo)
        if entry is None or entry[1] != key:
            return
        _forget_locked(lo)
    _release_range(lo, entry[0])


def _watch_host(tensors):
    """With the engine's host registration cache on (config host_register_cache_bytes > 0), the
    host memory of a keyed request may stay registered after the request. A registered range
    must leave the cache before its memory is freed, or a later tensor placed at the same address
    is taken for the old, unmapped pages (a device access through it faults; ADVICE r3, DESIGN
    §7). For every host tensor submitted while the cache is on:
      * a finalizer on its STORAGE object (torch keeps one Python object per live storage) hands
        the range to ddl_host_unregister when the storage dies — after its last view;
      * a recorded range that the tensor's storage now overlaps but does not match — the memory
        of a storage that was resized / re-set in place, or a range reused by a new storage — is
        unregistered before this submission can hit it in the cache."""
    lib = CPPBackend.c_api()
    if lib.ddl_get_config(b'host_register_cache_bytes') <= 0:
        return
    stale = []
    with _watched_lock:
        for t in tensors:
            if t.is_cuda:
                continue
            st = t.untyped_storage()
            lo, nbytes = st.data_ptr(), st.nbytes()
            if not lo or not nbytes:
                continue
            hi, key = lo + nbytes, id(st)
            e = _watched.get(lo)
            if e is not None and e[0] == hi and e[1] == key:
                continue  # recorded as it is: live storages never overlap, nothing else to check
            prev = _watched_by_storage.get(key)
            if prev is not None and prev != lo:  # this storage's memory moved (resize_ / set_)
                end, _, fin = _forget_locked(prev)
                fin.detach()
                stale.append((prev, end))
            i = max(0, bisect.bisect_right(_watched_starts, lo) - 1)
            while i < len(_watched_starts) and _watched_starts[i] < hi:
                start = _watched_starts[i]
                end, k, fin = _watched[start]
                if end > lo and (start, end, k) != (lo, hi, key):
                    _forget_locked(start)
                    fin.detach()
                    stale.append((start, end))
                    continue
                i += 1
            if lo not in _watched:
                fin = weakref.finalize(st, _on_storage_freed, lo, key)
                _watched[lo] = (hi, key, fin)
                _watched_by_storage[key] = lo
                bisect.insort(_watched_starts, lo)
    for a, b in stale:  # outside the lock: the engine may wait for its streams
        _release_range(a, b)


def _same_memory(a: torch.Tensor, b: torch.Tensor, what: str) -> int:
    ma, mb = memory_kind(a, f'{what} input'), memory_kind(b, f'{what} output')
    if ma != mb:
        raise ValueError(f'{what}: input and output must both be device or both be host tensors')
    return ma


def allreduce_async(tensor: torch.Tensor, name: str, communicator: Communicator = None,
                    output: torch.Tensor = None) -> Handle:
    """Register a keyed allreduce; returns a Handle.

    `name` plays the role of the TF op name: the same name on every rank identifies the same
    gradient, and only one request per name may be pending (TensorCommunicateRequest.h:21).
    Device tensors stay in HBM; host (CPU) tensors — the reference's only kind, its op is
    DEVICE_CPU (AllreduceOp.cc:68) — are fused through pinned staging to the GPU and back.
    """
    communicator = _comm(communicator)
    out = torch.empty_like(tensor) if output is None else output
    mem = _same_memory(tensor, out, 'allreduce_async')
    if mem == cb.MEMORY_HOST:
        _watch_host((tensor, out))
    # argument errors first: a group whose slot is never submitted would stay pending
    key, dt, stream = name.encode(), ddl_dtype(tensor), stream_handle_for(tensor)
    group = _Completion(1, (tensor, out))
    h = _NativeHandle(name, out, None, group, 0)  # the group holds the tensors
    st = CPPBackend.c_api().ddl_allreduce_submit_mem(
        communicator.id, key, tensor.data_ptr(), out.data_ptr(), tensor.numel(), dt, cb.OP_SUM, mem, stream,
        _native_done(), group.slots()[0])
    if st != cb.STATUS_OK:
        group.fail([0], st)
        check(st, 'ddl_allreduce_submit_mem')
    return h


def allreduce_async_batch(tensors, names, communicator: Communicator = None, outputs=None):
    """Register several keyed allreduces at once (one engine wake-up, one input-ready event);
    returns one Handle per tensor. Same key rules as `allreduce_async`; device and host tensors
    may be mixed (one submission per memory kind)."""
    import ctypes
    communicator = _comm(communicator)
    tensors = list(tensors)
    names = list(names)
    if len(tensors) != len(names):
        raise ValueError('one name per tensor')
    outputs = [torch.empty_like(t) for t in tensors] if outputs is None else list(outputs)
    k = len(tensors)
    if k == 0:
        return []
    in_place = all(o is t for t, o in zip(tensors, outputs))  # the DP wrapper's form
    mems = [memory_kind(t, 'allreduce_async_batch input') for t in tensors] if in_place else \
        [_same_memory(t, o, 'allreduce_async_batch') for t, o in zip(tensors, outputs)]
    # argument errors first: slots of a group that are never submitted would stay pending
    keys_all, dts_all = [n.encode() for n in names], [ddl_dtype(t) for t in tensors]
    if cb.MEMORY_HOST in mems:
        _watch_host([x for i, m in enumerate(mems) if m == cb.MEMORY_HOST for x in (tensors[i], outputs[i])])
    # one completion group for the batch: the engine completes every request natively (no
    # Python done() per tensor); the group keeps every tensor until the batch has completed, so
    # the handles hold only their outputs
    group = _Completion(k, (tensors, outputs))
    handles = [_NativeHandle(n, o, None, group, i) for i, (n, o) in enumerate(zip(names, outputs))]
    done, slots = _native_done(), group.slots()
    kinds = sorted(set(mems))
    for mem in kinds:
        if len(kinds) == 1:  # one memory kind (the usual batch): the arrays straight from the lists
            idx, ts, os_, ks, ds, users = range(k), tensors, outputs, keys_all, dts_all, slots
        else:
            idx = [i for i in range(k) if mems[i] == mem]
            ts, os_ = [tensors[i] for i in idx], [outputs[i] for i in idx]
            ks, ds = [keys_all[i] for i in idx], [dts_all[i] for i in idx]
            users = (ctypes.c_void_p * len(idx))(*[slots[i] for i in idx])
        m = len(idx)
        rest = [i for i in range(k) if mems[i] >= mem]  # this submission and the ones not made
        try:
            ins = (ctypes.c_void_p * m)(*[t.data_ptr() for t in ts])
            outs = ins if in_place else (ctypes.c_void_p * m)(*[o.data_ptr() for o in os_])
            st = CPPBackend.c_api().ddl_allreduce_submit_batch_mem(
                communicator.id, m, (ctypes.c_char_p * m)(*ks), ins, outs,
                (ctypes.c_size_t * m)(*[t.numel() for t in ts]), (ctypes.c_int * m)(*ds), cb.OP_SUM, mem,
                stream_handle_for(tensors[idx[0]]), done, users)
        except BaseException:
            group.fail(rest, _STATUS_ERROR_UNKNOWN)  # not submitted: no slot may stay pending
            raise
        if st != cb.STATUS_OK:
            group.fail(rest, st)
            check(st, 'ddl_allreduce_submit_batch_mem')
    return handles


def broadcast_async(tensor: torch.Tensor, name: str, root_rank: int, communicator: Communicator = None,
                    output: torch.Tensor = None) -> Handle:
    """Keyed broadcast (the TF op's asynchronous path, TensorBroadcastRequest): `output`
    (default: a new tensor; may be `tensor` itself) receives root's tensor. Device or host."""
    communicator = _comm(communicator)
    out = torch.empty_like(tensor) if output is None else output
    mem = _same_memory(tensor, out, 'broadcast_async')
    if mem == cb.MEMORY_HOST:
        _watch_host((tensor, out))
    key, dt, stream, root = name.encode(), ddl_dtype(tensor), stream_handle_for(tensor), int(root_rank)
    group = _Completion(1, (tensor, out))
    h = _NativeHandle(name, out, None, group, 0)  # the group holds the tensors
    st = CPPBackend.c_api().ddl_broadcast_submit_mem(
        communicator.id, key, tensor.data_ptr(), out.data_ptr(), tensor.numel(), dt, root, mem, stream,
        _native_done(), group.slots()[0])
    if st != cb.STATUS_OK:
        group.fail([0], st)
        check(st, 'ddl_broadcast_submit_mem')
    return h


class _GatherHandle(Handle):
    """Handle of a keyed allgather: the output is allocated by the engine's callback."""

    def __init__(self, key, tensor):
        super().__init__(key, None, tensor)
        self._shape_tail = tuple(tensor.shape[1:])
        self._dtype, self._device = tensor.dtype, tensor.device


_gathers = {}


@cb.ALLOC_FN
def _on_alloc(first_dim, nbytes, user):
    with _pending_lock:
        h = _gathers.get(user)
    if h is None:
        return None
    try:
        h.output = torch.empty((first_dim,) + h._shape_tail, dtype=h._dtype, device=h._device)
    except Exception:  # reported to the engine as an allocation failure
        return None
    return h.output.data_ptr() or None


@cb.DONE_FN
def _on_gather_done(status, user):
    with _pending_lock:
        h = _gathers.pop(user, None)
    if h is not None:
        h.status = status
        h._event.set()


def allgather_async(tensor: torch.Tensor, name: str, communicator: Communicator = None) -> Handle:
    """Keyed allgather (TensorAllgatherRequest): negotiated and fused with the other pending
    allgathers of the same dtype and memory kind; `handle.wait()` returns the gathered tensor
    (on the input's device: HBM, or host memory for a CPU tensor)."""
    communicator = _comm(communicator)
    src = tensor if tensor.dim() > 0 else tensor.reshape(1)
    mem = memory_kind(src, 'allgather_async input')
    row = 1
    for d in src.shape[1:]:
        row *= d
    uid = next(_ids)
    h = _GatherHandle(name, src)
    with _pending_lock:
        _gathers[uid] = h
    st = CPPBackend.c_api().ddl_allgather_submit_mem(
        communicator.id, name.encode(), src.data_ptr(), src.shape[0], row, ddl_dtype(src), mem,
        stream_handle_for(src), _on_alloc, _on_gather_done, uid)
    if st != cb.STATUS_OK:
        with _pending_lock:
            _gathers.pop(uid, None)
        check(st, 'ddl_allgather_submit_mem')
    return h


def broadcast_by_group(tensors, root_rank: int, communicator: Communicator = None, prefix: str = 'broadcast'):
    """Broadcast every tensor in place from `root_rank` as one negotiated, fused round of keyed
    requests (tensor_communicate.py:71-96: one Broadcast op per variable, assigned back)."""
    communicator = _comm(communicator)
    tensors = list(tensors)
    handles = [broadcast_async(t, f'{prefix}.{i:06d}', root_rank, communicator, output=t)
               for i, t in enumerate(tensors)]
    for h in handles:
        h.wait()
    return tensors


def broadcast_parameters(params, root_rank: int = 0, communicator: Communicator = None):
    """Initial weights from `root_rank` (the torch counterpart of broadcast_global_variables,
    tensor_communicate.py:111-129): `params` is a module's state_dict(), an iterable of
    (name, tensor) pairs, or an iterable of tensors; every tensor (device or host) is updated in
    place."""
    if hasattr(params, 'items'):
        items = sorted(params.items())
    else:
        items = list(params)
        if items and not isinstance(items[0], tuple):
            items = [(f'{i:06d}', t) for i, t in enumerate(items)]
    ts = [t.data if hasattr(t, 'data') else t for _, t in items]
    # device and host (CPU model) tensors alike, in place, as one negotiated round
    broadcast_by_group([t for t in ts if t.numel() > 0], root_rank, communicator, prefix='broadcast_parameters')
    return params


def synchronize(handle: Handle) -> torch.Tensor:
    return handle.wait()


def wait_all(communicator: Communicator = None) -> None:
    communicator = _comm(communicator)
    check(CPPBackend.c_api().ddl_wait_all(communicator.id), 'ddl_wait_all')
