#!/usr/bin/env python3
"""Where the host time of a keyed batch goes: the C5 set (4096 device buckets) submitted as one
batch at one rank, one_rank_shortcut on (no data plane) and off (pack -> allreduce -> unpack),
timing the submit call and the wait from Python; with log_level 2 the engine prints each round's
phases (take / enqueue / wait + done) on stderr.

    python tools/keyed_overhead.py > gpurun_out/keyed_overhead.jsonl 2> gpurun_out/keyed_overhead.err
"""
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault('ddl_lib', os.path.join(ROOT, 'experiment-distributed-deep-learning_amd', 'lib', 'libddl_amd_testing.so'))  # the testing build (raw kernels, test transport)
sys.path.insert(0, os.path.join(ROOT, 'experiment-distributed-deep-learning_amd'))


def main():
    import numpy as np
    import torch
    from ddl.torch.communicator import Communicator
    from ddl.torch.cpp_backend import DONE_FN, CPPBackend, check
    lib = CPPBackend.c_api()
    dev = torch.device('cuda', 0)
    torch.cuda.set_device(dev)
    comm = Communicator.world()
    rng = np.random.default_rng(5)
    k = 4096
    sizes = (np.exp(rng.uniform(np.log(4096), np.log(4 << 20), size=k)).astype(np.int64) // 256) * 256
    tensors, dts, keys = [], [], []
    for i in rng.permutation(k):
        half = rng.random() < 0.5
        tensors.append(torch.randn(int(sizes[i]) // (2 if half else 4), device=dev).to(torch.float16 if half else torch.float32))
        dts.append(19 if half else 1)
        keys.append(f'grad_{i:05d}'.encode())
    V = ctypes.c_void_p * k
    args = (k, (ctypes.c_char_p * k)(*keys), V(*[t.data_ptr() for t in tensors]), V(*[t.data_ptr() for t in tensors]),
            (ctypes.c_size_t * k)(*[t.numel() for t in tensors]), (ctypes.c_int * k)(*dts), 0,
            torch.cuda.current_stream(dev).cuda_stream, DONE_FN(), None)
    for shortcut in (1, 0):
        check(lib.ddl_set_config(b'one_rank_shortcut', shortcut), 'cfg')
        sub, wait = [], []
        for step in range(8):
            if step == 6:
                check(lib.ddl_set_config(b'log_level', 2), 'cfg')
            t0 = time.perf_counter()
            check(lib.ddl_allreduce_submit_batch(comm.id, *args), 'submit')
            t1 = time.perf_counter()
            check(lib.ddl_wait_all(comm.id), 'wait')
            t2 = time.perf_counter()
            sub.append((t1 - t0) * 1e6)
            wait.append((t2 - t1) * 1e6)
        check(lib.ddl_set_config(b'log_level', 0), 'cfg')
        sys.stderr.flush()
        print(json.dumps({'one_rank_shortcut': shortcut, 'submit_us': [round(x) for x in sub],
                          'wait_us': [round(x) for x in wait]}), flush=True)
    check(lib.ddl_set_config(b'one_rank_shortcut', 1), 'cfg')


if __name__ == '__main__':
    main()
