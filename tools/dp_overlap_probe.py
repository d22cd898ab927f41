#!/usr/bin/env python3
"""Does `overlap_backward` overlap? Two processes share the one GPU and run the whole N>1 engine
over the test-harness transport (point-to-point through gloo on host copies, tools/
gloo_transport.py — not xGMI): a data-parallel MLP step (8 x Linear(1024, 1024), batch 16384,
fp32) with the DP wrapper submitting every gradient at step() (overlap off) or from its backward
hook (overlap on). Two identically initialised replicas, interleaved rounds; rank 0 prints the
step times and checks both replicas stay equal.

    python tools/dp_overlap_probe.py > gpurun_out/dp_overlap.json
"""
import json
import os
import socket
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, 'experiment-distributed-deep-learning_amd'), os.path.join(ROOT, 'tools')):
    sys.path.insert(0, p)

WIDTH, LAYERS, BATCH, STEPS, ROUNDS = 1024, 8, 16384, 4, 3


def worker(rank, world, port, q):
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    import datetime

    import torch
    import torch.distributed as dist
    dist.init_process_group('gloo', rank=rank, world_size=world, timeout=datetime.timedelta(seconds=120))
    torch.cuda.set_device(0)
    import gloo_transport
    from ddl.torch.communicator import Communicator, finalize
    from ddl.torch.cpp_backend import CPPBackend
    from ddl.torch.parallelism.data import data_parallelism_distributed_optimizer_wrapper
    lib = CPPBackend.c_api()
    cbs = gloo_transport.init_world(lib, dist, torch, rank, world)  # noqa: F841 (keep alive)
    lib.ddl_set_config(b'tune', 0)
    comm = Communicator.world()

    def model_fn():
        torch.manual_seed(7)
        layers = []
        for _ in range(LAYERS):
            layers += [torch.nn.Linear(WIDTH, WIDTH), torch.nn.ReLU()]
        return torch.nn.Sequential(*layers).cuda()
    models = {False: model_fn(), True: model_fn()}
    opts = {ov: data_parallelism_distributed_optimizer_wrapper(torch.optim.SGD(m.parameters(), lr=1e-4), comm,
                                                               overlap_backward=ov) for ov, m in models.items()}
    g = torch.Generator(device='cuda').manual_seed(100 + rank)
    x = torch.randn(BATCH, WIDTH, device='cuda', generator=g)
    y = torch.randn(BATCH, WIDTH, device='cuda', generator=g)

    def step(ov):
        opts[ov].zero_grad()
        torch.nn.functional.mse_loss(models[ov](x), y).backward()
        opts[ov].step()

    times = {False: [], True: []}
    for ov in (False, True):  # warm-up (tuning-free: tune = 0)
        step(ov)
    torch.cuda.synchronize()
    for _ in range(ROUNDS):
        for ov in (False, True):
            dist.barrier()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(STEPS):
                step(ov)
            torch.cuda.synchronize()
            times[ov].append((time.perf_counter() - t0) / STEPS * 1e3)
    same = all(torch.equal(a, b) for a, b in zip(models[False].parameters(), models[True].parameters()))
    dist.barrier()
    finalize()
    q.put((rank, times, same))


def main():
    import torch.multiprocessing as mp
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        port = s.getsockname()[1]
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    world = 2
    procs = [ctx.Process(target=worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict((r, (t, same)) for r, t, same in (q.get(timeout=600) for _ in range(world)))
    for p in procs:
        p.join(timeout=30)
    t, same = res[0]
    grad_mib = LAYERS * (WIDTH * WIDTH + WIDTH) * 4 / 2 ** 20
    print(json.dumps({'probe': 'dp_overlap_backward', 'ranks': world, 'transport': 'test harness: gloo over host copies',
                      'model': f'{LAYERS} x Linear({WIDTH},{WIDTH}) fp32, batch {BATCH}', 'grad_MiB': round(grad_mib, 1),
                      'ms_per_step_overlap_off': [round(v, 2) for v in t[False]],
                      'ms_per_step_overlap_on': [round(v, 2) for v in t[True]],
                      'replicas_equal': same}), flush=True)


if __name__ == '__main__':
    main()
