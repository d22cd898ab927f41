"""Helpers between torch tensors and the C-ABI (reference counterpart: src/py/ddl/tensorflow/util.py)."""
import torch

from ddl.torch import cpp_backend as cb

_DTYPES = {
    torch.float32: cb.DT_FLOAT,
    torch.float64: cb.DT_DOUBLE,
    torch.int32: cb.DT_INT32,
    torch.int64: cb.DT_INT64,
    torch.float16: cb.DT_HALF,
    torch.bfloat16: cb.DT_BFLOAT16,
}
if hasattr(torch, 'uint64'):
    _DTYPES[torch.uint64] = cb.DT_UINT64


def ddl_dtype(t: torch.Tensor) -> int:
    try:
        return _DTYPES[t.dtype]
    except KeyError:
        raise TypeError(f'ddl: unsupported dtype {t.dtype} '
                        f'(supported: {sorted(str(d) for d in _DTYPES)})') from None


def current_stream_handle(device=None) -> int:
    """hipStream_t of torch's current stream (0 = legacy default stream)."""
    return torch.cuda.current_stream(device).cuda_stream


def memory_kind(t: torch.Tensor, what: str = 'tensor') -> int:
    """ddl_memory of a contiguous tensor: device (HBM) or host (the reference's CPU tensors)."""
    if not t.is_contiguous():
        raise ValueError(f'{what} must be contiguous')
    return cb.MEMORY_DEVICE if t.is_cuda else cb.MEMORY_HOST


def stream_handle_for(t: torch.Tensor) -> int:
    """The submitter's stream for a device tensor; 0 for host tensors (ready at submission)."""
    return current_stream_handle(t.device) if t.is_cuda else 0


def require_device_tensor(t: torch.Tensor, what: str = 'tensor') -> None:
    if not t.is_cuda:
        raise ValueError(f'{what} must be a device (HBM) tensor')
    if not t.is_contiguous():
        raise ValueError(f'{what} must be contiguous')
