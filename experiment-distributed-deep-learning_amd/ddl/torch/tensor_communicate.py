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
import itertools
import threading

import torch

from ddl.torch import cpp_backend as cb
from ddl.torch.communicator import Communicator
from ddl.torch.cpp_backend import CPPBackend, check
from ddl.torch.util import current_stream_handle, ddl_dtype, require_device_tensor


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


_pending = {}
_pending_lock = threading.Lock()
_ids = itertools.count(1)


@cb.DONE_FN
def _on_done(status, user):
    with _pending_lock:
        h = _pending.pop(user, None)
    if h is not None:
        h.status = status
        h._event.set()


def allreduce_async(tensor: torch.Tensor, name: str, communicator: Communicator = None,
                    output: torch.Tensor = None) -> Handle:
    """Register a keyed allreduce of a device tensor; returns a Handle.

    `name` plays the role of the TF op name: the same name on every rank identifies the same
    gradient, and only one request per name may be pending (TensorCommunicateRequest.h:21).
    """
    communicator = _comm(communicator)
    require_device_tensor(tensor, 'allreduce_async input')
    out = torch.empty_like(tensor) if output is None else output
    require_device_tensor(out, 'allreduce_async output')
    uid = next(_ids)
    h = Handle(name, out, (tensor, out))
    with _pending_lock:
        _pending[uid] = h
    st = CPPBackend.c_api().ddl_allreduce_submit(
        communicator.id, name.encode(), tensor.data_ptr(), out.data_ptr(), tensor.numel(),
        ddl_dtype(tensor), cb.OP_SUM, current_stream_handle(tensor.device), _on_done, uid)
    if st != cb.STATUS_OK:
        with _pending_lock:
            _pending.pop(uid, None)
        check(st, 'ddl_allreduce_submit')
    return h


def allreduce_async_batch(tensors, names, communicator: Communicator = None, outputs=None):
    """Register several keyed allreduces at once (one engine wake-up, one input-ready event);
    returns one Handle per tensor. Same key rules as `allreduce_async`."""
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
    for t, o in zip(tensors, outputs):
        require_device_tensor(t, 'allreduce_async_batch input')
        require_device_tensor(o, 'allreduce_async_batch output')
    uids = [next(_ids) for _ in range(k)]
    handles = [Handle(n, o, (t, o)) for n, t, o in zip(names, tensors, outputs)]
    with _pending_lock:
        _pending.update(zip(uids, handles))
    keys = (ctypes.c_char_p * k)(*[n.encode() for n in names])
    ins = (ctypes.c_void_p * k)(*[t.data_ptr() for t in tensors])
    outs = (ctypes.c_void_p * k)(*[o.data_ptr() for o in outputs])
    ns = (ctypes.c_size_t * k)(*[t.numel() for t in tensors])
    dts = (ctypes.c_int * k)(*[ddl_dtype(t) for t in tensors])
    users = (ctypes.c_void_p * k)(*uids)
    st = CPPBackend.c_api().ddl_allreduce_submit_batch(
        communicator.id, k, keys, ins, outs, ns, dts, cb.OP_SUM, current_stream_handle(tensors[0].device),
        _on_done, users)
    if st != cb.STATUS_OK:
        with _pending_lock:
            for u in uids:
                _pending.pop(u, None)
        check(st, 'ddl_allreduce_submit_batch')
    return handles


def broadcast_async(tensor: torch.Tensor, name: str, root_rank: int, communicator: Communicator = None,
                    output: torch.Tensor = None) -> Handle:
    """Keyed broadcast (the TF op's asynchronous path, TensorBroadcastRequest): `output`
    (default: a new tensor; may be `tensor` itself) receives root's tensor."""
    communicator = _comm(communicator)
    require_device_tensor(tensor, 'broadcast_async input')
    out = torch.empty_like(tensor) if output is None else output
    require_device_tensor(out, 'broadcast_async output')
    uid = next(_ids)
    h = Handle(name, out, (tensor, out))
    with _pending_lock:
        _pending[uid] = h
    st = CPPBackend.c_api().ddl_broadcast_submit(
        communicator.id, name.encode(), tensor.data_ptr(), out.data_ptr(), tensor.numel(), ddl_dtype(tensor),
        int(root_rank), current_stream_handle(tensor.device), _on_done, uid)
    if st != cb.STATUS_OK:
        with _pending_lock:
            _pending.pop(uid, None)
        check(st, 'ddl_broadcast_submit')
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
    allgathers of the same dtype; `handle.wait()` returns the gathered tensor."""
    communicator = _comm(communicator)
    require_device_tensor(tensor, 'allgather_async input')
    src = tensor if tensor.dim() > 0 else tensor.reshape(1)
    row = 1
    for d in src.shape[1:]:
        row *= d
    uid = next(_ids)
    h = _GatherHandle(name, src)
    with _pending_lock:
        _gathers[uid] = h
    st = CPPBackend.c_api().ddl_allgather_submit(
        communicator.id, name.encode(), src.data_ptr(), src.shape[0], row, ddl_dtype(src),
        current_stream_handle(src.device), _on_alloc, _on_gather_done, uid)
    if st != cb.STATUS_OK:
        with _pending_lock:
            _gathers.pop(uid, None)
        check(st, 'ddl_allgather_submit')
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
    (name, tensor) pairs, or an iterable of tensors; device tensors are updated in place."""
    if hasattr(params, 'items'):
        items = sorted(params.items())
    else:
        items = list(params)
        if items and not isinstance(items[0], tuple):
            items = [(f'{i:06d}', t) for i, t in enumerate(items)]
    ts = [t.data if hasattr(t, 'data') else t for _, t in items]
    dev = [t for t in ts if t.is_cuda and t.numel() > 0]
    broadcast_by_group(dev, root_rank, communicator, prefix='broadcast_parameters')
    for t in ts:
        if not t.is_cuda and t.numel() > 0:
            t.copy_(broadcast(t, root_rank, communicator))
    return params


def synchronize(handle: Handle) -> torch.Tensor:
    return handle.wait()


def wait_all(communicator: Communicator = None) -> None:
    communicator = _comm(communicator)
    check(CPPBackend.c_api().ddl_wait_all(communicator.id), 'ddl_wait_all')
