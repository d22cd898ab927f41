"""Small-bucket behaviour of the per-hop reduce (measurement tool, not shipped): back-to-back
launches of acc += in for 4 KiB .. 64 MiB fp32 per cache-policy variant, interleaved rounds,
best of 3. Prints one JSON object per size.

    python tools/small_sweep.py [--sets 3]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'experiment-distributed-deep-learning_amd'))


def main():
    import torch
    from ddl.torch.cpp_backend import CPPBackend, check
    ap = argparse.ArgumentParser()
    ap.add_argument('--sets', type=int, default=3)
    a = ap.parse_args()
    lib = CPPBackend.c_api()
    dev = torch.device('cuda', 0)
    s = torch.cuda.current_stream(dev)
    sh = s.cuda_stream
    variants = {'plain': 0, 'nt_a': 1, 'nt_all': 7}
    for size in [4 << 10, 64 << 10, 256 << 10, 1 << 20, 2 << 20, 4 << 20, 16 << 20, 64 << 20]:
        m = size // 4
        bufs = [(torch.zeros(m, device=dev), torch.ones(m, device=dev)) for _ in range(a.sets)]
        reps = int(min(2000, max(20, (256 << 20) // size)))
        best = {k: float('inf') for k in variants}
        for _ in range(3):
            for k, v in variants.items():
                for i in range(3):
                    x, y = bufs[i % a.sets]
                    check(lib.ddl_reduce_sum2_variant(v, x.data_ptr(), x.data_ptr(), y.data_ptr(), m, 1, sh), 'r')
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(s)
                for i in range(reps):
                    x, y = bufs[i % a.sets]
                    check(lib.ddl_reduce_sum2_variant(v, x.data_ptr(), x.data_ptr(), y.data_ptr(), m, 1, sh), 'r')
                e1.record(s)
                torch.cuda.synchronize()
                best[k] = min(best[k], e0.elapsed_time(e1) / reps * 1e3)
        print(json.dumps({'bytes': size, 'us': {k: round(v, 2) for k, v in best.items()},
                          'hbm_GBs': {k: round(3 * size / v / 1e3, 1) for k, v in best.items()}}), flush=True)
        del bufs


if __name__ == '__main__':
    main()
