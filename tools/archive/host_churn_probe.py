"""Is the pageable keyed host batch's slow D2H phase tied to tensor churn? Four legs of the C5
set as pageable host tensors through the keyed path (3 steps each), either on the SAME tensors
every leg (`keep`) or on a fresh 2.45 GB set per leg with the last one freed (`churn`); one
process per mode (measurement)."""
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'experiment-distributed-deep-learning_amd'))
import torch  # noqa: E402

from ddl.torch.communicator import Communicator  # noqa: E402
from ddl.torch.cpp_backend import DONE_FN, MEMORY_HOST, CPPBackend, check  # noqa: E402


def make_set(k=4096, seed=5):
    rng = np.random.default_rng(seed)
    sizes = (np.exp(rng.uniform(np.log(4096), np.log(4 << 20), size=k)).astype(np.int64) // 256) * 256
    ts, dts = [], []
    for i in rng.permutation(k):
        half = rng.random() < 0.5
        n = int(sizes[i]) // (2 if half else 4)
        ts.append(torch.randn(n).to(torch.float16 if half else torch.float32))
        dts.append(19 if half else 1)
    return ts, dts


def main(mode):
    lib = CPPBackend.c_api()
    torch.cuda.set_device(0)
    comm = Communicator.world()
    check(lib.ddl_set_config(b'one_rank_shortcut', 0), 'cfg')
    ts, dts = make_set()
    for leg in range(4):
        if mode == 'churn' and leg:
            del ts
            ts, dts = make_set(seed=5 + leg)
        k = len(ts)
        keys = (ctypes.c_char_p * k)(*[f'c{leg}_{i:05d}'.encode() for i in range(k)])
        ptrs = (ctypes.c_void_p * k)(*[t.data_ptr() for t in ts])
        args = (k, keys, ptrs, ptrs, (ctypes.c_size_t * k)(*[t.numel() for t in ts]), (ctypes.c_int * k)(*dts), 0,
                MEMORY_HOST, None, DONE_FN(), None)
        ms = []
        for _ in range(4):
            t0 = time.perf_counter()
            check(lib.ddl_allreduce_submit_batch_mem(comm.id, *args), 'submit')
            check(lib.ddl_wait_all(comm.id), 'wait')
            ms.append(round((time.perf_counter() - t0) * 1e3, 1))
        print(json.dumps({'mode': mode, 'leg': leg, 'step_ms': ms}), flush=True)


if __name__ == '__main__':
    main(sys.argv[1])
