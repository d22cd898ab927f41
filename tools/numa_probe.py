"""Host side of the keyed host-tensor path vs CPU placement (measurement tool, not
shipped). Prints the box's NUMA layout, the GPU's node, this process's allowed CPUs, then runs the
C5 host batch (bench.keyed_host_c5) with the main thread pinned to a CPU set chosen before the
engine starts a thread (its handler thread and memcpy workers inherit it) and before the host
tensors are allocated (first touch):
    python tools/numa_probe.py topo
    python tools/numa_probe.py run {default|nobind|local|remote} [threads]
One JSON line per run."""
import ctypes
import glob
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault('ddl_lib', os.path.join(ROOT, 'experiment-distributed-deep-learning_amd', 'lib', 'libddl_amd_testing.so'))  # the testing build (raw kernels, test transport)


def parse_list(s):
    out = set()
    for part in s.strip().split(','):
        if not part:
            continue
        a, _, b = part.partition('-')
        out.update(range(int(a), int(b or a) + 1))
    return out


def nodes():
    res = {}
    for p in sorted(glob.glob('/sys/devices/system/node/node[0-9]*')):
        try:
            res[int(p.rsplit('node', 1)[1])] = parse_list(open(os.path.join(p, 'cpulist')).read())
        except OSError:
            pass
    return res


def gpu_node():
    """NUMA node of GPU 0's PCI function (torch's device properties; no second HIP runtime)."""
    import torch
    p = torch.cuda.get_device_properties(0)
    bdf = f'{getattr(p, "pci_domain_id", 0):04x}:{getattr(p, "pci_bus_id", 0):02x}:{getattr(p, "pci_device_id", 0):02x}.0'
    try:
        return bdf, int(open(f'/sys/bus/pci/devices/{bdf}/numa_node').read())
    except OSError:
        return bdf, None


def topo():
    allowed = os.sched_getaffinity(0)
    ns = nodes()
    print(json.dumps({'nproc': os.cpu_count(), 'allowed': len(allowed), 'gpu': gpu_node(),
                      'allowed_by_node': {n: len(c & allowed) for n, c in ns.items()},
                      'node_sizes': {n: len(c) for n, c in ns.items()}}), flush=True)


def run(mode, threads):
    allowed = os.sched_getaffinity(0)
    ns = nodes()
    bdf, gnode = gpu_node()
    pick = allowed
    if mode in ('local', 'remote') and gnode is not None and ns:
        local = ns.get(gnode, set()) & allowed
        remote = (set().union(*[c for n, c in ns.items() if n != gnode]) & allowed)
        pick = local if mode == 'local' else remote
    if not pick:
        print(json.dumps({'mode': mode, 'skipped': 'no allowed CPU in that set'}), flush=True)
        return
    os.sched_setaffinity(0, pick)
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, 'experiment-distributed-deep-learning_amd'))
    import numpy as np
    import torch
    import bench
    from ddl.torch.communicator import Communicator
    from ddl.torch.cpp_backend import CPPBackend, check
    torch.cuda.set_device(0)
    lib = CPPBackend.c_api()
    # 'nobind': the default CPU set with the engine's own NUMA binding off (host_numa_bind 0, set
    # before the handler starts), to A/B the binding against 'default'
    check(lib.ddl_set_config(b'host_numa_bind', 0 if mode == 'nobind' else 1), 'cfg')
    comm = Communicator.world()
    check(lib.ddl_set_config(b'host_copy_threads', threads), 'cfg')
    # raw rates of the pieces, on the same CPUs: one memcpy stream pageable -> pinned, and pinned
    # H2D / D2H of 256 MiB on one stream
    src = np.random.default_rng(0).standard_normal(1 << 26).astype(np.float32)
    pin = torch.empty(1 << 26, pin_memory=True)
    dst = pin.numpy()
    np.copyto(dst, src)
    t0 = time.perf_counter()
    for _ in range(4):
        np.copyto(dst, src)
    memcpy_gbs = 4 * src.nbytes / (time.perf_counter() - t0) / 1e9
    dev = torch.empty(1 << 26, device='cuda')
    dev.copy_(pin, non_blocking=True)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(4):
        dev.copy_(pin, non_blocking=True)
    torch.cuda.synchronize()
    h2d = 4 * src.nbytes / (time.perf_counter() - t0) / 1e9
    t0 = time.perf_counter()
    for _ in range(4):
        pin.copy_(dev, non_blocking=True)
    torch.cuda.synchronize()
    d2h = 4 * src.nbytes / (time.perf_counter() - t0) / 1e9
    r = bench.keyed_host_c5(lib, comm, steps=3)
    rp = bench.keyed_host_c5(lib, comm, steps=3, pinned=True)
    print(json.dumps({'mode': mode, 'cpus': len(pick), 'gpu_bdf': bdf, 'gpu_node': gnode,
                      'host_copy_threads': threads, 'memcpy_1thread_GBs': round(memcpy_gbs, 1),
                      'h2d_GBs': round(h2d, 1), 'd2h_GBs': round(d2h, 1), 'keyed_host_c5_ms': r['ms'],
                      'keyed_host_c5_GiBs': r['bucket_GiBs'], 'engine_thread': r['engine_thread'],
                      'keyed_host_c5_pinned_ms': rp['ms'], 'pinned_engine_thread': rp['engine_thread']}), flush=True)


if __name__ == '__main__':
    if sys.argv[1] == 'topo':
        topo()
    else:
        run(sys.argv[2], int(sys.argv[3]) if len(sys.argv) > 3 else 7)
