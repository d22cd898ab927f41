"""Keyed host C5 batch (bench.keyed_host_c5, pageable tensors) with the main thread — which
allocates and first-touches the tensors — left where the OS put it vs bound to the CPUs of the
GPU's NUMA node (the engine's own threads are bound either way: host_numa_bind). Interleaved
rounds; reports where the tensors' pages landed (move_pages query) (measurement)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'experiment-distributed-deep-learning_amd'))
sys.path.insert(0, os.path.join(ROOT, 'tools'))
import torch  # noqa: E402

import bench  # noqa: E402
from ddl.torch.communicator import Communicator  # noqa: E402
from ddl.torch.cpp_backend import CPPBackend  # noqa: E402
from host_numa_ab import cpulist, gpu_node  # noqa: E402

lib = CPPBackend.c_api()
torch.cuda.set_device(0)
comm = Communicator.world()
node = gpu_node()
allowed = os.sched_getaffinity(0)
local = cpulist(open(f'/sys/devices/system/node/node{node}/cpulist').read()) & allowed
print(json.dumps({'gpu_node': node, 'allowed': len(allowed), 'local': len(local),
                  'main_thread_cpu_now': os.sched_getaffinity(0) == local}), flush=True)
for rep in range(3):
    for bind in (False, True):
        if bind:
            os.sched_setaffinity(0, local)
        r = bench.keyed_host_c5(lib, comm, steps=3)
        os.sched_setaffinity(0, allowed)
        print(json.dumps({'rep': rep, 'bind': bind, 'ms': r['ms'], 'pack_ms': r['engine_thread']['pack_ms'],
                          'unpack_ms': r['engine_thread']['unpack_ms'], 'warm': r['warmup_steps_ms'],
                          'cgroup': r['cgroup_cpu']}), flush=True)
