"""Data-parallel training callbacks for torch loops (mirrors of the reference's Keras callbacks):

* InitialParametersBroadcast — initial_paramerters_broadcast.py:9-42: before the first batch,
  the root rank's model (and optimizer) state is broadcast to every rank, so replicas start
  identical.
* MetricAverage — metric_average_callback.py:9-59: at epoch end every metric is averaged over
  the ranks (allreduce / size), metrics in sorted name order so every rank issues the same
  sequence of collectives; skipped at size 1 (:56-59).
* LearningRateSchedule / LearningRateWarmup — lr_warm_up_callback.py:6-124: the learning rate
  of a torch optimizer scaled per batch (or per epoch: staircase) by a multiplier of the epoch,
  with momentum correction; the warm-up ramps from lr / size to lr over `warmup_epochs`. No
  communication: only the communicator's size and rank are read.

The first two go through the engine's keyed requests (one negotiated, fused round per call).
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


class LearningRateSchedule:
    """Mirror of LearningRateScheduleCallback (lr_warm_up_callback.py:6-93) for a torch optimizer.

    Call the hooks from the training loop as Keras calls them: `on_train_begin()` once,
    `on_epoch_begin(epoch)`, `on_batch_begin(batch)` / `on_batch_end(batch)` around every step,
    `on_epoch_end(epoch, logs)`. Between `start_epoch` and `end_epoch` every parameter group's lr
    is `initial_lr * multiplier(epoch)` — at the first batch of an epoch with `staircase`, else
    at every batch with the fractional epoch `epoch + batch / steps_per_epoch`.

    `momentum_correction` (Goyal et al.; reference :58-66) scales a group's momentum by
    new_lr / old_lr for the one batch whose lr changed and restores it after. It exists for
    optimizers that keep the lr INSIDE the velocity, as Keras' SGD does (v = m*v - lr*g): there an
    lr change would otherwise reach the step only gradually. torch's SGD keeps it outside
    (buf = m*buf + g; p -= lr*buf), so an lr change takes effect at once and rescaling the momentum
    would change the dynamics instead of preserving them. Default None = automatic: on
    only for an optimizer that declares `lr_scaled_velocity = True`; every torch.optim optimizer
    gets no correction — which is what the reference's correction achieves on Keras. True forces
    it (an optimizer that stores lr-scaled velocity without declaring it), False turns it off.

    `initial_lr`: None takes each group's lr at `on_train_begin` (the reference reads the
    optimizer's single lr); a number sets every group from it. `steps_per_epoch`: needed unless
    staircase; `on_train_begin(params=...)` may detect it from Keras-style params ('steps', or
    'samples' and 'batch_size', :29-43)."""

    def __init__(self, optimizer, multiplier, start_epoch=0, end_epoch=None, staircase=True,
                 momentum_correction=None, steps_per_epoch=None, initial_lr=None):
        self.optimizer = optimizer
        self.start_epoch = start_epoch
        self.end_epoch = end_epoch
        self.staircase = staircase
        if momentum_correction is None:
            momentum_correction = bool(getattr(optimizer, 'lr_scaled_velocity', False))
        self.momentum_correction = momentum_correction
        self.initial_lr = initial_lr
        self.restore_momentum = None
        self.steps_per_epoch = steps_per_epoch
        self.current_epoch = None
        if not callable(multiplier):  # a constant multiplier changes only at epoch boundaries (:24-26)
            self.staircase = True
            self.multiplier = lambda epoch: multiplier
        else:
            self.multiplier = multiplier

    def _autodetect_steps_per_epoch(self, params):
        params = params or {}
        if params.get('steps'):
            return params['steps']
        if params.get('samples') and params.get('batch_size'):
            return params['samples'] // params['batch_size']
        raise ValueError('Could not autodetect the number of steps per epoch. Please specify the steps_per_epoch '
                         f'parameter to the {self.__class__.__name__}().')

    def _adjust_learning_rate(self, epoch):
        factor = self.multiplier(epoch)
        self.restore_momentum = None
        for i, group in enumerate(self.optimizer.param_groups):
            old_lr = group['lr']
            new_lr = self.initial_lr[i] * factor
            group['lr'] = new_lr
            if self.momentum_correction and 'momentum' in group and old_lr:
                if self.restore_momentum is None:
                    self.restore_momentum = {}
                self.restore_momentum[i] = group['momentum']
                group['momentum'] = group['momentum'] * new_lr / old_lr

    def _restore_momentum_if_needed(self):
        if self.restore_momentum:
            for i, m in self.restore_momentum.items():
                self.optimizer.param_groups[i]['momentum'] = m
            self.restore_momentum = None

    def on_train_begin(self, logs=None, params=None):
        groups = self.optimizer.param_groups
        if self.initial_lr is None:
            self.initial_lr = [g['lr'] for g in groups]
        elif not isinstance(self.initial_lr, (list, tuple)):
            self.initial_lr = [self.initial_lr] * len(groups)
        if not self.staircase and not self.steps_per_epoch:
            self.steps_per_epoch = self._autodetect_steps_per_epoch(params)

    def on_epoch_begin(self, epoch, logs=None):
        self.current_epoch = epoch

    def on_batch_begin(self, batch, logs=None):
        if self.current_epoch < self.start_epoch or (self.end_epoch is not None and
                                                     self.current_epoch >= self.end_epoch):
            return
        if self.staircase and batch == 0:
            self._adjust_learning_rate(self.current_epoch)
        elif not self.staircase:
            self._adjust_learning_rate(self.current_epoch + float(batch) / self.steps_per_epoch)

    def on_batch_end(self, batch, logs=None):
        self._restore_momentum_if_needed()

    def on_epoch_end(self, epoch, logs=None):
        if logs is not None:
            logs['lr'] = self.optimizer.param_groups[0]['lr']
        return logs


class LearningRateWarmup(LearningRateSchedule):
    """Mirror of LearningRateWarmupCallback (lr_warm_up_callback.py:96-124): over the first
    `warmup_epochs` the lr rises linearly from initial_lr / size to initial_lr, per batch:
    multiplier(e) = 1 / size * ((e + 1 / steps_per_epoch) * (size - 1) / warmup_epochs + 1), with
    e the fractional epoch. The scripts scale the base lr by the size first (the reference's
    examples/data_parallelism.py:73-101). `verbose` prints only on rank 0."""

    def __init__(self, optimizer, warmup_epochs=5, momentum_correction=None, steps_per_epoch=None, verbose=0,
                 initial_lr=None, communicator: Communicator = None):
        comm = Communicator.world() if communicator is None else communicator

        def multiplier(epoch):
            # shifted by one batch so each epoch ends on a round number (:106-109)
            epoch += 1. / self.steps_per_epoch
            return 1. / comm.size * (epoch * (comm.size - 1) / warmup_epochs + 1)

        super().__init__(optimizer, multiplier, start_epoch=0, end_epoch=warmup_epochs, staircase=False,
                         momentum_correction=momentum_correction, steps_per_epoch=steps_per_epoch,
                         initial_lr=initial_lr)
        self.verbose = verbose if comm.rank == 0 else 0

    def on_epoch_end(self, epoch, logs=None):
        logs = super().on_epoch_end(epoch, logs)
        if epoch == self.end_epoch - 1 and self.verbose > 0:
            print('\nEpoch %d: finished gradual learning rate warmup to %g.' %
                  (epoch + 1, self.optimizer.param_groups[0]['lr']))
        return logs
