"""Tensor collectives (mirror of reference src/py/ddl/tensorflow/tensor_communicate.py:9-42).

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

    Sparse gradients (the reference's IndexedSlices -> allgather branch, :26-30) need the
    allgather collective, which is not part of this engine yet.
    """
    communicator = _comm(communicator)
    if tensor.is_sparse:
        raise NotImplementedError('sparse gradients need allgather (not implemented in ddl_amd)')
    summed = allreduce(tensor, communicator)
    if return_mean:
        summed.div_(communicator.size)
    return summed


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
            raise TimeoutError(f'allreduce request {self.key!r} did not complete')
        self._keep = None
        if self.status != cb.STATUS_OK:
            raise cb.DDLError(self.status, f'allreduce request {self.key!r}', '')
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


def synchronize(handle: Handle) -> torch.Tensor:
    return handle.wait()


def wait_all(communicator: Communicator = None) -> None:
    communicator = _comm(communicator)
    check(CPPBackend.c_api().ddl_wait_all(communicator.id), 'ddl_wait_all')
