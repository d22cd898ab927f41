"""Keyed host C5 batch (bench.keyed_host_c5: pageable and pinned tensors) with the copy threads'
plain memcpy vs non-temporal stores (config host_copy_nt), interleaved rounds (measurement)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'experiment-distributed-deep-learning_amd'))
import torch  # noqa: E402

import bench  # noqa: E402
from ddl.torch.communicator import Communicator  # noqa: E402
from ddl.torch.cpp_backend import CPPBackend  # noqa: E402

lib = CPPBackend.c_api()
torch.cuda.set_device(0)
comm = Communicator.world()
threads = [int(t) for t in os.environ.get('AB_THREADS', '7').split(',')]
for rep in range(3):
    for pinned in (False, True):
        for th in threads:
            for nt in (0, 1):
                r = bench.keyed_host_c5(lib, comm, steps=3, pinned=pinned,
                                        settings={'host_copy_nt': nt, 'host_copy_threads': th})
                print(json.dumps({'rep': rep, 'pinned': pinned, 'threads': th, 'nt': nt, 'ms': r['ms'],
                                  'pack_ms': r['engine_thread']['pack_ms'], 'unpack_ms': r['engine_thread']['unpack_ms'],
                                  'slot_wait_ms': r['engine_thread']['slot_wait_ms'],
                                  'warm': r['warmup_steps_ms']}), flush=True)
