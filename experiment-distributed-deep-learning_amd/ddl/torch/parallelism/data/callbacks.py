"""Data-parallel training callbacks for torch loops (mirrors of the reference's Keras callbacks):

* InitialParametersBroadcast — initial_paramerters_broadcast.py:9-42: before the first batch,
  the root rank's model (and optimizer) state is broadcast to every rank, so replicas start
  identical.
* MetricAverage — metric_average_callback.py:9-59: at epoch end every metric is averaged over
  the ranks (allreduce / size), metrics in sorted name order so every rank issues the same
  sequence of collectives; skipped at size 1 (:56-59).

Both go through the engine's keyed requests (one negotiated, fused round per call).
"""
import torch

from ddl.torch.communicator import Communicator
from ddl.torch.tensor_communicate import allreduce_async, broadcast_parameters


class InitialParametersBroadcast:
    """Call `on_batch_begin()` from the training loop (or `broadcast()` once)."""

    def __init__(self, model: torch.nn.Module, root_rank: int = 0, optimizer: torch.optim.Optimizer = None,
                 communicator: Communicator = None):
        self._model, self._optimizer = model, optimizer
        self._root = root_rank
        self._comm = Communicator.world() if communicator is None else communicator
        self._done = False

    def broadcast(self):
        broadcast_parameters(self._model.state_dict(), self._root, self._comm)
        if self._optimizer is not None:
            state = []
            for gi, group in enumerate(self._optimizer.param_groups):
                for pi, p in enumerate(group['params']):
                    for k, v in sorted(self._optimizer.state.get(p, {}).items()):
                        if torch.is_tensor(v) and v.numel() > 0:
                            state.append((f'opt.{gi}.{pi}.{k}', v))
            if state:
                broadcast_parameters(state, self._root, self._comm)
        self._done = True

    def on_batch_begin(self, batch=None, logs=None):
        if not self._done:
            self.broadcast()


class MetricAverage:
    """`on_epoch_end(epoch, logs)` replaces every value in `logs` by its mean over the ranks."""

    def __init__(self, communicator: Communicator = None, device=None):
        self._comm = Communicator.world() if communicator is None else communicator
        self._device = torch.device('cuda', torch.cuda.current_device()) if device is None else device

    def average(self, logs: dict) -> dict:
        if not logs:
            return logs
        names = sorted(logs)
        vals = [torch.as_tensor(logs[k], dtype=torch.float64).reshape(1).to(self._device) for k in names]
        handles = [allreduce_async(v, f'MetricAverage.{k}', self._comm) for k, v in zip(names, vals)]
        for k, h in zip(names, handles):
            logs[k] = h.wait().item() / self._comm.size
        return logs

    def on_epoch_end(self, epoch=None, logs=None):
        if self._comm.size > 1:
            self.average(logs)
        return logs
