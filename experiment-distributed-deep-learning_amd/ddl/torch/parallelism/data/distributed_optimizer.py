"""Data-parallel optimizer wrapper for torch.optim (mirror of reference
src/py/ddl/tensorflow/keras/parallelism/data/distributed_optimizer.py:9-110).

Every rank computes gradients on its shard of the batch; before the wrapped optimizer's
`step()` each gradient is submitted as a keyed allreduce request (the reference builds one
`Allreduce` op per gradient, :43-68), the engine negotiates and fuses them, and the sum is
divided by the communicator size (allreduce_gradient, tensor_communicate.py:21-25). A sparse
gradient (torch sparse COO, TF's IndexedSlices) goes through allreduce_gradient's allgather
branch (:26-30), as the reference's wrapper does for every grad. At size 1 nothing is
communicated (the reference's `tf.cond(size > 1)`, :53-60).

CPU models (the reference's deployment: its op is CPU-only, AllreduceOp.cc:68): with
`pin_host_gradients` (default) each dense CPU gradient is moved once into pinned memory and
kept there — zero_grad() zeroes it in place instead of dropping it, and autograd accumulates
into it in place — so the engine's unpack kernel writes the reduced gradients straight into
them over PCIe (no D2H copy, no host memcpy).

Overlap with backward (`overlap_backward=True`): a post-accumulate-grad hook on every parameter
submits its keyed allreduce the moment autograd has finished its gradient, so the engine
negotiates and reduces the late layers' gradients while the early layers' are still being
computed (the reference's graph lets TF schedule each Allreduce op as soon as its input exists);
step() only waits for them. The keys count backwards from the last parameter and the fusion
plans are capped at `bucket_bytes`, so a round's plans run in backward order, each as soon as its
own gradients are ready (DDP-style buckets). Gradient accumulation over several backward passes:
run all but the last inside `no_sync()`, as with torch DDP.
"""
import contextlib
import functools

import torch

from ddl.torch.communicator import Communicator
from ddl.torch.tensor_communicate import allreduce_async, allreduce_async_batch, allreduce_gradient


class DataParallelismDistributedOptimizer:
    """Mixin placed in front of the wrapped optimizer class (the reference's approach)."""
    communicator: Communicator = None
    pin_host_gradients: bool = True
    _ddl_name = 'DataParallelismDistributedOptimizer'
    _grad_handles = None  # overlap_backward: param -> Handle submitted by its hook
    _syncing = True

    def _key(self, gi: int, pi: int) -> str:
        return f'{self._ddl_name}/{type(self).__name__}/Allreduce/group{gi}/param{pi:05d}'

    def _comm(self) -> Communicator:
        return self.communicator or Communicator.world()

    def _register_overlap_hooks(self) -> None:
        # keys numbered from the last parameter back: the engine runs a round's plans in key
        # order, so the plans holding the gradients autograd produces first go first, each
        # waiting only for its own gradients (a sequential model's backward runs in reverse
        # parameter order)
        self._grad_handles = {}
        params = [p for group in self.param_groups for p in group['params'] if p.requires_grad]
        self._hooks = [
            p.register_post_accumulate_grad_hook(functools.partial(
                self._grad_ready, f'{self._ddl_name}/{type(self).__name__}/Allreduce/backward{len(params) - 1 - i:05d}'))
            for i, p in enumerate(params)]

    def _grad_ready(self, key: str, p: torch.Tensor) -> None:
        g = p.grad
        if not self._syncing or g is None or g.is_sparse or not g.is_contiguous() or self._comm().size <= 1:
            return  # no_sync, or left to step() (sparse / strided gradients)
        if p in self._grad_handles:
            raise RuntimeError(f'{key}: gradient accumulated again while its allreduce is pending; run the '
                               'earlier backward passes inside no_sync()')
        if self._pinning() and not g.is_cuda and not g.is_pinned():
            p.grad = g = g.pin_memory()
        self._grad_handles[p] = allreduce_async(g, key, self._comm(), output=g)

    @contextlib.contextmanager
    def no_sync(self):
        """Backward passes inside accumulate gradients without reducing them (overlap_backward)."""
        old, self._syncing = self._syncing, False
        try:
            yield
        finally:
            self._syncing = old

    def _drain_hooked(self) -> dict:
        handles, self._grad_handles = (self._grad_handles or {}), ({} if self._grad_handles is not None else None)
        return handles

    def _pinning(self) -> bool:
        return self.pin_host_gradients and torch.cuda.is_available()

    @staticmethod
    def _pinned_host_grad(g) -> bool:
        return g is not None and not g.is_cuda and not g.is_sparse and g.is_pinned()

    def allreduce_gradients(self) -> None:
        comm = self._comm()
        if comm.size <= 1:
            return
        # gradients already submitted by the backward hooks (overlap_backward)
        hooked = self._drain_hooked()
        for p, h in hooked.items():
            h.wait().div_(comm.size)
        pin = self._pinning()
        params, grads, keys, sparse = [], [], [], []
        for gi, group in enumerate(self.param_groups):
            for pi, p in enumerate(group['params']):
                if p.grad is None or p in hooked:
                    continue
                if p.grad.is_sparse:
                    sparse.append(p)
                    continue
                if pin and not p.grad.is_cuda and p.grad.is_contiguous() and not p.grad.is_pinned():
                    p.grad = p.grad.pin_memory()  # once: zero_grad keeps it (see below)
                params.append(p)
                grads.append(p.grad if p.grad.is_contiguous() else p.grad.contiguous())
                keys.append(self._key(gi, pi))
        # one keyed request per gradient (the reference builds one Allreduce op per grad,
        # distributed_optimizer.py:50-63), registered as one batch, reduced in place
        handles = zip(params, allreduce_async_batch(grads, keys, comm, outputs=grads))
        for p, h in handles:
            out = h.wait()
            out.div_(comm.size)
            if out.data_ptr() != p.grad.data_ptr():
                p.grad.copy_(out)
        # sparse gradients: every rank's rows gathered, values averaged (same order on all ranks)
        for p in sparse:
            p.grad = allreduce_gradient(p.grad, comm)

    def zero_grad(self, set_to_none: bool = True) -> None:
        # pinned host gradients survive zero_grad (zeroed in place), so the next backward
        # accumulates into the same pinned buffers
        for h in self._drain_hooked().values():  # reductions of gradients about to be dropped
            h.wait()
        keep = []
        if self._pinning():
            keep = [(p, p.grad) for group in self.param_groups for p in group['params']
                    if self._pinned_host_grad(p.grad)]
        super().zero_grad(set_to_none)
        with torch.no_grad():
            for p, g in keep:
                if p.grad is None:
                    g.zero_()
                    p.grad = g

    @torch.no_grad()
    def step(self, closure=None):
        self.allreduce_gradients()
        return super().step(closure)

    @property
    def is_distributed_optimizer(self) -> bool:
        return True


def data_parallelism_distributed_optimizer_wrapper(
        optimizer: torch.optim.Optimizer,
        communicator: Communicator = None,
        pin_host_gradients: bool = True,
        overlap_backward: bool = False,
        bucket_bytes: int = 32 << 20) -> torch.optim.Optimizer:
    """Return an optimizer of a subclass of `type(optimizer)` whose step() first averages the
    gradients across `communicator` (default: the world). Parameter groups and state are
    shared with `optimizer`. `pin_host_gradients`: keep CPU gradients in pinned memory;
    `overlap_backward`: submit each gradient's allreduce from a backward hook (module
    docstring) and cap the engine's fusion plans at `bucket_bytes` (the engine-wide
    `fusion_threshold_bytes`, so every rank must build the wrapper the same way; None keeps the
    configured cap): a round's gradients then reduce as several plans in backward order, each
    starting once its own gradients exist."""
    opt_cls = optimizer.__class__
    assert issubclass(opt_cls, torch.optim.Optimizer)
    cls = type(opt_cls.__name__, (DataParallelismDistributedOptimizer, opt_cls), {})
    res = cls.__new__(cls)
    res.__dict__.update(optimizer.__dict__)
    res.communicator = communicator
    res.pin_host_gradients = pin_host_gradients
    if overlap_backward:
        if bucket_bytes:
            from ddl.torch import config
            config.set('fusion_threshold_bytes', int(bucket_bytes))
        res._register_overlap_hooks()
    return res
