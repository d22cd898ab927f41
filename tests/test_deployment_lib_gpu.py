"""The deployment library (lib/libddl_amd.so, exactly include/ddl_amd.h) on the GPU, on its own.

The rest of the suite drives the testing build (conftest.py: the same engine objects plus the
test surface). Here a fresh process loads ONLY libddl_amd.so through the torch mirror — as a
training script would — and runs what one GPU can run of the product path: the world
communicator (ddl_init_single), device and host allreduce, the grouped allreduce, the keyed path
with its data plane forced (pack kernel -> allreduce -> unpack kernel, pinned host chunks for
CPU tensors), broadcast / allgather, the kernel-timing hooks. Integer-valued data, so every
result is exact; the process checks from /proc/self/maps that the testing build never loaded.
"""
import os
import subprocess
import sys

import pytest

from conftest import DEPLOYMENT_LIB, PKG

SCRIPT = r'''
import os, sys
sys.path.insert(0, PKG)
import torch
from ddl.torch.cpp_backend import CPPBackend, check
from ddl.torch import config
from ddl.torch.communicator import Communicator
from ddl.torch.tensor_communicate import (allgather, allreduce, allreduce_, allreduce_async_batch, allreduce_batch_,
                                          broadcast)
lib = CPPBackend.c_api()
assert CPPBackend.path() == DEPLOYMENT_LIB and not CPPBackend.has_testing_api()
assert not hasattr(lib, 'ddl_reduce_local') and not hasattr(lib, 'ddl_init_test_transport')
comm = Communicator.world()
assert comm.size == 1 and comm.rank == 0
g = torch.Generator().manual_seed(7)
x = torch.randint(-1000, 1000, (1_000_003,), generator=g).float()
# device: allreduce (a new tensor), in place, grouped
d = x.cuda()
assert torch.equal(allreduce(d, comm).cpu(), x)
assert torch.equal(allreduce_(d.clone(), comm).cpu(), x)
bs = [x[:4099].cuda().half(), x[:300].cuda().half(), x[:65537].cuda().half()]
allreduce_batch_(bs, comm)
assert all(torch.equal(b.cpu().float(), x[:b.numel()]) for b in bs)
# host: the chunked H2D -> allreduce -> D2H pipeline
assert torch.equal(allreduce(x, comm), x)
# the keyed path with its data plane forced at one rank: pack -> allreduce -> unpack, device and
# host tensors (pageable and pinned), several plans
old = {k: config.get(k) for k in ('one_rank_shortcut', 'fusion_threshold_bytes', 'host_chunk_bytes')}
config.set('one_rank_shortcut', 0)
config.set('fusion_threshold_bytes', 1 << 20)
config.set('host_chunk_bytes', 256 << 10)
try:
    parts = [x[i * 50_000:(i + 1) * 50_000 + i] for i in range(12)]
    dev = [p.cuda() for p in parts] + [p.cuda().double() for p in parts[:3]]
    host = [p.clone() for p in parts] + [parts[0].clone().pin_memory(), parts[1].half()]
    hs = allreduce_async_batch(dev, [f'd{i}' for i in range(len(dev))], comm, outputs=[torch.empty_like(t) for t in dev])
    hh = allreduce_async_batch(host, [f'h{i}' for i in range(len(host))], comm, outputs=host)
    for t, h in zip(dev, hs):
        assert torch.equal(h.wait(), t)
    want = [p.clone() for p in parts] + [parts[0], parts[1].half()]
    for w, h in zip(want, hh):
        assert torch.equal(h.wait(), w)
finally:
    for k, v in old.items():
        config.set(k, v)
# broadcast / allgather (tensor_communicate.py's other collectives)
assert torch.equal(broadcast(d, 0, comm).cpu(), x)
assert torch.equal(allgather(d[:1000].reshape(100, 10), comm).cpu(), x[:1000].reshape(100, 10))
maps = open('/proc/self/maps').read()
assert 'libddl_amd.so' in maps and 'libddl_amd_testing.so' not in maps, 'the testing build was loaded'
print('deployment library ok')
'''


@pytest.mark.gpu
def test_deployment_library_alone_on_the_gpu():
    env = dict(os.environ)
    env.pop('ddl_lib', None)  # the torch mirror's default: lib/libddl_amd.so
    code = f'PKG = {PKG!r}\nDEPLOYMENT_LIB = {DEPLOYMENT_LIB!r}\n' + SCRIPT
    p = subprocess.run([sys.executable, '-c', code], env=env, capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, (p.stdout[-2000:], p.stderr[-4000:])
    assert 'deployment library ok' in p.stdout
