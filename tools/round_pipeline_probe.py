#!/usr/bin/env python3
"""Pipelined keyed rounds at one rank, data plane on (one_rank_shortcut = 0): a stream of keyed
submits — one request per call, so the engine runs many small rounds back to back — timed from
the first submit to ddl_wait_all, with pipeline_rounds 1 (a completion thread fires done() while
the engine thread takes and enqueues the next round) and 0 (each round waited for first).
Also a DDP-style bucket stream: B buckets of S bytes submitted as separate batches.

    python tools/round_pipeline_probe.py > gpurun_out/round_pipeline.jsonl
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
    import torch
    from ddl.torch.communicator import Communicator
    from ddl.torch.cpp_backend import DONE_FN, CPPBackend, check
    lib = CPPBackend.c_api()
    dev = torch.device('cuda', 0)
    torch.cuda.set_device(dev)
    comm = Communicator.world()
    stream = torch.cuda.current_stream(dev).cuda_stream
    check(lib.ddl_set_config(b'one_rank_shortcut', 0), 'cfg')
    nodone = DONE_FN()
    for count, nbytes, per_batch in ((256, 64 << 10, 1), (64, 4 << 20, 1), (16, 32 << 20, 1), (32, 1 << 20, 8)):
        ts = [torch.randn(nbytes // 4, device=dev) for _ in range(count)]
        res = {}
        for pipelined in (1, 0, 1, 0):
            check(lib.ddl_set_config(b'pipeline_rounds', pipelined), 'cfg')
            best = None
            for rep in range(5):
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for b in range(0, count, per_batch):
                    k = min(per_batch, count - b)
                    V = ctypes.c_void_p * k
                    keys = (ctypes.c_char_p * k)(*[f'p{rep}_{b + j:05d}'.encode() for j in range(k)])
                    ptrs = V(*[ts[b + j].data_ptr() for j in range(k)])
                    check(lib.ddl_allreduce_submit_batch(comm.id, k, keys, ptrs, ptrs,
                                                         (ctypes.c_size_t * k)(*[ts[b + j].numel() for j in range(k)]),
                                                         (ctypes.c_int * k)(*([1] * k)), 0, stream, nodone, None),
                          'submit')
                check(lib.ddl_wait_all(comm.id), 'wait')
                dt = (time.perf_counter() - t0) * 1e3
                best = dt if best is None else min(best, dt)
            res.setdefault(pipelined, []).append(round(best, 3))
        print(json.dumps({'buckets': count, 'bucket_bytes': nbytes, 'per_submit': per_batch,
                          'ms_pipelined': res[1], 'ms_unpipelined': res[0],
                          'us_per_bucket_pipelined': round(min(res[1]) * 1e3 / count, 1),
                          'us_per_bucket_unpipelined': round(min(res[0]) * 1e3 / count, 1)}), flush=True)
    check(lib.ddl_set_config(b'pipeline_rounds', 1), 'cfg')
    check(lib.ddl_set_config(b'one_rank_shortcut', 1), 'cfg')


if __name__ == '__main__':
    main()
