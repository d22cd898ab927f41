#!/usr/bin/env python3
"""A/B of the keyed host allreduce's unpack on the C5 bucket set (4096 host buckets, 2.45 GB),
interleaved in one process so box-to-box noise cancels: pageable tensors (staged both ways),
pinned tensors staged both ways (host_zero_copy = 0), pinned tensors with the unpack kernel
writing the results over PCIe (host_zero_copy = 1). One rank, data plane forced.

    python tools/host_unpack_ab.py > gpurun_out/host_unpack_ab.jsonl
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'experiment-distributed-deep-learning_amd'))


def main():
    import statistics

    import torch

    import bench
    from ddl.torch.communicator import Communicator
    from ddl.torch.cpp_backend import CPPBackend
    lib = CPPBackend.c_api()
    torch.cuda.set_device(0)
    comm = Communicator.world()
    res = {'pageable': [], 'pinned_staged': [], 'pinned_device_unpack': []}
    for rnd in range(4):
        for name in res:
            lib.ddl_set_config(b'host_zero_copy', 0 if name == 'pinned_staged' else 1)
            r = bench.keyed_host_c5(lib, comm, steps=2, pinned=name != 'pageable')
            res[name].append(r['ms'])
            print(json.dumps({'round': rnd, 'case': name, 'ms': r['ms'],
                              'device_unpack_plans_per_step': r['device_unpack_plans_per_step']}), flush=True)
    lib.ddl_set_config(b'host_zero_copy', 1)
    print(json.dumps({'summary': {k: {'best_ms': min(v), 'median_ms': statistics.median(v)} for k, v in res.items()},
                      'bytes': 2446361088, 'host_copy_threads': lib.ddl_get_config(b'host_copy_threads'),
                      'host_chunk_bytes': lib.ddl_get_config(b'host_chunk_bytes')}), flush=True)


if __name__ == '__main__':
    main()
