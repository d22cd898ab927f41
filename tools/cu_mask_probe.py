"""How many CUs the HBM-bound kernels need (measurement): the run-form fold (one P = 8
chunk, 32 MiB fp32), the C4 fp16 fold (2 MiB chunk) and the 256 MiB two-input reduce, each timed on
streams created with hipExtStreamCreateWithCUMask for masks enabling fewer CUs. At N > 1 the fold
overlaps RCCL's send / recv kernels, which need CUs of their own to drive the xGMI links: if the
fold keeps its rate on fewer CUs, the engine can leave some to RCCL. Two mask shapes: the lowest k
bits set ('low'), and k bits spread evenly over the 256 ('spread').
    python tools/cu_mask_probe.py"""
import ctypes
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault('ddl_lib', os.path.join(ROOT, 'experiment-distributed-deep-learning_amd', 'lib', 'libddl_amd_testing.so'))  # the testing build (raw kernels, test transport)
sys.path.insert(0, os.path.join(ROOT, 'experiment-distributed-deep-learning_amd'))
sys.path.insert(0, os.path.join(ROOT, 'tests'))
from ddl.torch.cpp_backend import CPPBackend, check  # noqa: E402
from _helpers import hip_runtime  # noqa: E402


def masked_stream(hip, ncu, enabled):
    words = (ncu + 31) // 32
    m = (ctypes.c_uint32 * words)()
    for c in enabled:
        m[c // 32] |= 1 << (c % 32)
    s = ctypes.c_void_p()
    assert hip.hipExtStreamCreateWithCUMask(ctypes.byref(s), words, m) == 0
    return s


def main():
    lib = CPPBackend.c_api()
    hip = hip_runtime()
    f = hip.hipExtStreamCreateWithCUMask
    f.restype, f.argtypes = ctypes.c_int, [ctypes.POINTER(ctypes.c_void_p), ctypes.c_uint32, ctypes.c_void_p]
    f = hip.hipStreamDestroy
    f.restype, f.argtypes = ctypes.c_int, [ctypes.c_void_p]
    dev = torch.device('cuda', 0)
    torch.cuda.set_device(dev)
    ncu = torch.cuda.get_device_properties(0).multi_processor_count
    P = ctypes.c_void_p * 7
    fold32 = [[torch.rand(8 << 20, device=dev) for _ in range(9)] for _ in range(2)]
    fold16 = [[torch.rand(1 << 20, device=dev).half() for _ in range(9)] for _ in range(1)]
    fold8m = [[torch.rand(2 << 20, device=dev) for _ in range(9)] for _ in range(2)]  # 8 MiB: the tile form
    red = [(torch.rand(64 << 20, device=dev), torch.rand(64 << 20, device=dev)) for _ in range(3)]
    # the fusion pack / unpack on the C5 set (4096 segments of 4 KiB - 4 MiB, bench.fusion_c5's sizes)
    import numpy as np
    rng = np.random.default_rng(5)
    sizes = (np.exp(rng.uniform(np.log(4096), np.log(4 << 20), size=4096)).astype(np.int64) // 256) * 256
    segs = [torch.empty(int(x), dtype=torch.uint8, device=dev) for x in sizes]
    flat = torch.empty(int(sizes.sum()) + 256 * 4096, dtype=torch.uint8, device=dev)
    sptr = (ctypes.c_void_p * 4096)(*[t.data_ptr() for t in segs])
    sbytes = (ctypes.c_size_t * 4096)(*[int(x) for x in sizes])

    def run(kind, k, sh):
        if kind in ('pack', 'unpack'):
            if kind == 'pack':
                check(lib.ddl_pack(flat.data_ptr(), sptr, sbytes, 4096, sh), 'pack')
            else:
                check(lib.ddl_unpack(sptr, flat.data_ptr(), sbytes, 4096, sh), 'unpack')
            return 2 * int(sizes.sum())
        if kind == 'reduce':
            a, b = red[k % 3]
            check(lib.ddl_reduce_local(a.data_ptr(), b.data_ptr(), a.numel(), 1, sh), 'reduce')
            return 3 * a.numel() * 4
        bufs, dt = ((fold32[k % 2], 1) if kind == 'fold_fp32_32MiB' else (fold8m[k % 2], 1) if kind == 'fold_fp32_8MiB'
                    else (fold16[0], 19))
        n = bufs[0].numel()
        check(lib.ddl_reduce_fold_ordered(bufs[8].data_ptr(), bufs[0].data_ptr(), P(*[t.data_ptr() for t in bufs[1:8]]),
                                          7, n, dt, 1 if dt == 1 else 0, sh), 'fold')
        return 9 * n * bufs[0].element_size()

    # 'every m-th off': CU c disabled when c % m == m - 1 (the masks a reserve for RCCL would use)
    cases = [('full', list(range(ncu)))] + [(f'every {m}th off', [c for c in range(ncu) if c % m != m - 1])
                                            for m in (16, 8, 4, 2)] + [('low 224', list(range(224)))]
    for shape, enabled in cases:
        k = len(enabled)
        if True:
            s = masked_stream(hip, ncu, enabled)
            ts = torch.cuda.ExternalStream(s.value)
            res = {}
            for kind, reps in (('fold_fp32_32MiB', 20), ('fold_fp32_8MiB', 40), ('fold_fp16_2MiB', 50), ('reduce', 12),
                               ('pack', 4), ('unpack', 4)):
                for i in range(3):
                    run(kind, i, s.value)
                best = 1e9
                for _ in range(3):
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record(ts)
                    byts = 0
                    for i in range(reps):
                        byts = run(kind, i, s.value)
                    e1.record(ts)
                    torch.cuda.synchronize()
                    best = min(best, e0.elapsed_time(e1) / reps / 1e3)
                res[kind] = {'us': round(best * 1e6, 2), 'TBps': round(byts / best / 1e12, 3)}
            print(json.dumps({'shape': shape, 'cus_enabled': k, **res}), flush=True)
            hip.hipStreamDestroy(s)


if __name__ == '__main__':
    main()
