#!/usr/bin/env python3
"""Does `overlap_backward` overlap? Two processes share the one GPU and run the whole N>1 engine
over the test-harness transport (point-to-point through gloo on host copies, tools/
gloo_transport.py — not xGMI): a data-parallel MLP step (8 x Linear(1024, 1024), batch 16384,
fp32) with the DP wrapper submitting every gradient at step() (overlap off) or from its backward
hook in 8 MiB buckets (overlap on; the cap applies to both replicas' fusion plans). Two
identically initialised replicas, interleaved rounds; rank 0 prints the step times, the compute
and the allreduce alone, and whether both replicas stay equal.

    python tools/dp_overlap_probe.py > gpurun_out/dp_overlap.json
"""
import json
import os
import socket
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault('ddl_lib', os.path.join(ROOT, 'experiment-distributed-deep-learning_amd', 'lib', 'libddl_amd_testing.so'))  # the testing build (raw kernels, test transport)
for p in (os.path.join(ROOT, 'experiment-distributed-deep-learning_amd'), os.path.join(ROOT, 'tools')):
    sys.path.insert(0, p)

WIDTH, LAYERS, BATCH, STEPS, ROUNDS, BUCKET = 1024, 8, 16384, 4, 3, 8 << 20


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
    # overlap on: 8 MiB buckets (two layers' gradients per plan), set before any step
    opts = {ov: data_parallelism_distributed_optimizer_wrapper(torch.optim.SGD(m.parameters(), lr=1e-4), comm,
                                                               overlap_backward=ov, bucket_bytes=BUCKET)
            for ov, m in models.items()}
    g = torch.Generator(device='cuda').manual_seed(100 + rank)
    x = torch.randn(BATCH, WIDTH, device='cuda', generator=g)
    y = torch.randn(BATCH, WIDTH, device='cuda', generator=g)

    def step(ov):
        opts[ov].zero_grad()
        torch.nn.functional.mse_loss(models[ov](x), y).backward()
        opts[ov].step()

    plain = model_fn()  # the same step without any communication (compute alone)
    plain_opt = torch.optim.SGD(plain.parameters(), lr=1e-4)

    def step_plain():
        plain_opt.zero_grad()
        torch.nn.functional.mse_loss(plain(x), y).backward()
        plain_opt.step()

    from ddl.torch.tensor_communicate import allreduce_async_batch
    grads = [p.grad.clone() if p.grad is not None else torch.zeros_like(p) for p in models[False].parameters()]

    def step_comm():  # the gradients' allreduce alone (one batch)
        for h in allreduce_async_batch(grads, [f'comm_only/{i}' for i in range(len(grads))], comm, outputs=grads):
            h.wait()

    times = {False: [], True: [], 'compute_only': [], 'comm_only': []}
    for ov in (False, True):  # warm-up (tuning-free: tune = 0)
        step(ov)
    step_plain()
    step_comm()
    torch.cuda.synchronize()
    lib.ddl_set_config(b'log_level', 2)  # the engine's round lines of one overlapped step
    # host timeline of that step: when the hooks submit, when backward() returns, when the GPU
    # has finished the backward (an event on the default stream), when step() returns
    marks = []
    hook_ts = []
    orig = opts[True]._grad_ready
    def stamped(key, p):
        hook_ts.append(time.perf_counter())
        orig(key, p)
    opts[True]._grad_ready = stamped
    for h in opts[True]._hooks:
        h.remove()
    opts[True]._register_overlap_hooks()
    opts[True].zero_grad()
    t0 = time.perf_counter()
    loss = torch.nn.functional.mse_loss(models[True](x), y)
    ev = torch.cuda.Event()
    loss.backward()
    marks.append(('backward_returned', time.perf_counter()))
    ev.record()
    opts[True].step()
    marks.append(('step_returned', time.perf_counter()))
    ev.synchronize()
    marks.append(('gpu_backward_done_seen', time.perf_counter()))
    torch.cuda.synchronize()
    lib.ddl_set_config(b'log_level', 0)
    opts[True]._grad_ready = orig
    for h in opts[True]._hooks:
        h.remove()
    opts[True]._register_overlap_hooks()
    step(False)  # the other replica takes the same number of steps
    timeline = {'first_hook_ms': round((hook_ts[0] - t0) * 1e3, 2), 'last_hook_ms': round((hook_ts[-1] - t0) * 1e3, 2),
                'hooks': len(hook_ts)}
    timeline.update({k: round((v - t0) * 1e3, 2) for k, v in marks})
    for _ in range(ROUNDS):
        for name, fn in (('compute_only', step_plain), ('comm_only', step_comm)):
            dist.barrier()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(STEPS):
                fn()
            torch.cuda.synchronize()
            times[name].append((time.perf_counter() - t0) / STEPS * 1e3)
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
    q.put((rank, times, same, timeline))


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
    res = dict((r, (t, same, tl)) for r, t, same, tl in (q.get(timeout=600) for _ in range(world)))
    for p in procs:
        p.join(timeout=30)
    t, same, tl = res[0]
    grad_mib = LAYERS * (WIDTH * WIDTH + WIDTH) * 4 / 2 ** 20
    print(json.dumps({'probe': 'dp_overlap_backward', 'ranks': world, 'transport': 'test harness: gloo over host copies',
                      'model': f'{LAYERS} x Linear({WIDTH},{WIDTH}) fp32, batch {BATCH}', 'grad_MiB': round(grad_mib, 1),
                      'ms_per_step_overlap_off': [round(v, 2) for v in t[False]],
                      'ms_per_step_overlap_on': [round(v, 2) for v in t[True]],
                      'ms_compute_only': [round(v, 2) for v in t['compute_only']],
                      'ms_allreduce_only': [round(v, 2) for v in t['comm_only']],
                      'replicas_equal': same, 'rank0_timeline_ms': tl}), flush=True)


if __name__ == '__main__':
    main()
