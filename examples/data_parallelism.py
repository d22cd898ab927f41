"""Data-parallel training with the engine: the torch counterpart of the reference's
src/py/ddl/examples/data_parallelism.py (Keras + its MPI path), line for line in structure:

  * every rank takes its shard of the data (get_processing_data, :47-53);
  * the learning rate is scaled by the world size, and warmed up to it over `--warmup_epochs`
    (LearningRateWarmup, the reference's LearningRateWarmupCallback, :73-101);
  * the optimizer is wrapped so every step averages the gradients over the ranks through keyed,
    fused allreduces (data_parallelism_distributed_optimizer_wrapper, :80-84);
  * rank 0's initial weights are broadcast (InitialParametersBroadcast, :91-93), and the epoch's
    metrics are averaged over the ranks (MetricAverage, :95).

The datasets cannot be downloaded here, so the data is synthetic with MNIST's / CIFAR-10's shapes
(28x28x1 / 32x32x3 inputs, 10 classes), a fixed random linear labelling to learn.

    python -m torch.distributed.run --nproc-per-node 8 examples/data_parallelism.py --epochs 3
    python examples/data_parallelism.py --epochs 1 --samples 2048      (one process)
"""
import os
import sys
from argparse import ArgumentParser

import torch
import torch.nn as nn

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                'experiment-distributed-deep-learning_amd'))


def parse():
    p = ArgumentParser()
    p.add_argument('--dataset', default='mnist', choices=('mnist', 'cifar10'))
    p.add_argument('--batch_size', default=128, type=int)
    p.add_argument('--epochs', default=20, type=int)
    p.add_argument('--warmup_epochs', default=5, type=int)
    p.add_argument('--lr', default=0.001, type=float)
    p.add_argument('--samples', default=60000, type=int, help='synthetic training samples (all ranks)')
    return p.parse_args()


def model_for(dataset):
    c, hw = (1, 28) if dataset == 'mnist' else (3, 32)
    side = ((hw - 2 - 2) // 2)
    return nn.Sequential(nn.Conv2d(c, 32, 3), nn.ReLU(), nn.Conv2d(32, 64, 3), nn.ReLU(), nn.MaxPool2d(2),
                         nn.Dropout(0.25), nn.Flatten(), nn.Linear(64 * side * side, 128), nn.ReLU(),
                         nn.Dropout(0.5), nn.Linear(128, 10)), (c, hw)


def synthetic(samples, shape, seed=0):
    g = torch.Generator().manual_seed(seed)
    x = torch.rand((samples,) + shape, generator=g)
    w = torch.randn(x[0].numel(), 10, generator=g)
    return x, (x.flatten(1) @ w).argmax(1)


def get_processing_data(data, communicator):
    """This rank's shard (reference examples/data_parallelism.py:47-53): equal contiguous shares of
    len(data) // size samples in rank order, the remainder going to the last rank."""
    share = len(data) // communicator.size
    lo = share * communicator.rank
    hi = len(data) if communicator.rank + 1 == communicator.size else lo + share
    return data[lo:hi]


def main():
    args = parse()
    from ddl.torch.communicator import Communicator
    from ddl.torch.parallelism.data import (InitialParametersBroadcast, LearningRateWarmup, MetricAverage,
                                            data_parallelism_distributed_optimizer_wrapper)
    world = Communicator.world()
    dev = torch.device('cuda', torch.cuda.current_device())
    model, (c, hw) = model_for(args.dataset)
    model = model.to(dev)
    x, y = synthetic(args.samples, (c, hw, hw))
    x_train, y_train = get_processing_data(x, world), get_processing_data(y, world)
    # scale the lr by the number of replicas; the warm-up ramps to it from slightly above base_lr
    scaled_lr = world.size * args.lr
    optimizer = data_parallelism_distributed_optimizer_wrapper(torch.optim.Adam(model.parameters(), lr=scaled_lr),
                                                               world)
    if world.size > 1:
        InitialParametersBroadcast(model, 0, optimizer, communicator=world).broadcast()
    steps = max(1, len(x_train) // args.batch_size)
    warmup = LearningRateWarmup(optimizer, warmup_epochs=args.warmup_epochs, steps_per_epoch=steps,
                                initial_lr=scaled_lr, verbose=1, communicator=world)
    average = MetricAverage(world, device=dev)
    loss_fn = nn.CrossEntropyLoss()
    warmup.on_train_begin()
    history = []
    for epoch in range(args.epochs):
        warmup.on_epoch_begin(epoch)
        model.train()
        total, correct, seen = 0.0, 0, 0
        perm = torch.randperm(len(x_train), generator=torch.Generator().manual_seed(epoch))
        for b in range(steps):
            idx = perm[b * args.batch_size:(b + 1) * args.batch_size]
            xb, yb = x_train[idx].to(dev), y_train[idx].to(dev)
            warmup.on_batch_begin(b)
            optimizer.zero_grad()
            out = model(xb)
            loss = loss_fn(out, yb)
            loss.backward()
            optimizer.step()
            warmup.on_batch_end(b)
            total += loss.item() * len(idx)
            correct += int((out.argmax(1) == yb).sum())
            seen += len(idx)
        logs = warmup.on_epoch_end(epoch, {'loss': total / seen, 'accuracy': correct / seen})
        logs = average.on_epoch_end(epoch, logs)
        history.append(logs)
        if world.rank == 0:
            print(f'epoch {epoch + 1}/{args.epochs}: ' + ', '.join(f'{k} {v:.4g}' for k, v in sorted(logs.items())),
                  flush=True)
    return history


if __name__ == '__main__':
    main()
