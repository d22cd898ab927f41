#!/usr/bin/env python3
"""Probe for the keyed host path over pinned host tensors: what HIP reports for
torch's pinned CPU tensors, and how fast the fusion pack / unpack kernels (k_seg_tiles) move the
C5 bucket set when they read and write those tensors directly over PCIe (no host memcpy),
next to the DMA engines' rate for one large pinned buffer.

    python tools/zero_copy_probe.py > gpurun_out/zero_copy.jsonl

The kernels are launched on host pointers only after hipPointerGetAttributes has shown every
one of them to be pinned host memory mapped at the same address on the device (otherwise the
probe prints the attributes and stops)."""
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault('ddl_lib', os.path.join(ROOT, 'experiment-distributed-deep-learning_amd', 'lib', 'libddl_amd_testing.so'))  # the testing build (raw kernels, test transport)
sys.path.insert(0, os.path.join(ROOT, 'experiment-distributed-deep-learning_amd'))


class PtrAttr(ctypes.Structure):
    _fields_ = [('type', ctypes.c_int), ('device', ctypes.c_int), ('devicePointer', ctypes.c_void_p),
                ('hostPointer', ctypes.c_void_p), ('isManaged', ctypes.c_int), ('allocationFlags', ctypes.c_uint)]


RANGE_START, RANGE_SIZE = 11, 12  # hipPointer_attribute


def attrs(hip, p):
    a = PtrAttr()
    rc = hip.hipPointerGetAttributes(ctypes.byref(a), ctypes.c_void_p(p))
    start, size = ctypes.c_void_p(), ctypes.c_size_t()
    rs = hip.hipPointerGetAttribute(ctypes.byref(start), RANGE_START, ctypes.c_void_p(p))
    rz = hip.hipPointerGetAttribute(ctypes.byref(size), RANGE_SIZE, ctypes.c_void_p(p))
    if rc or rs or rz:
        hip.hipGetLastError()  # a failed query (pageable memory) must not leave a sticky error
    return {'rc': rc, 'type': a.type, 'dev': a.devicePointer, 'host': a.hostPointer, 'flags': a.allocationFlags,
            'range_rc': (rs, rz), 'range_start': start.value, 'range_size': size.value}


def emit(d):
    print(json.dumps(d), flush=True)


def main():
    import numpy as np
    import torch
    from ddl.torch.cpp_backend import CPPBackend, check
    lib = CPPBackend.c_api()
    hip = ctypes.CDLL('libamdhip64.so')
    dev = torch.device('cuda', 0)
    torch.cuda.set_device(dev)

    # 1. what HIP says about torch's pinned tensors and about pageable ones
    pin = torch.empty(1 << 20, dtype=torch.float32, pin_memory=True)
    page = torch.empty(1 << 20, dtype=torch.float32)
    p = pin.data_ptr()
    emit({'probe': 'attrs', 'pinned': attrs(hip, p), 'pinned_interior': attrs(hip, p + 4096),
          'pageable': attrs(hip, page.data_ptr()), 'pinned_ptr': p})

    # 2. the C5 set (4096 buckets, log-uniform 4 KiB - 4 MiB, fp32 / fp16) as pinned tensors
    rng = np.random.default_rng(5)
    k = 4096
    sizes = (np.exp(rng.uniform(np.log(4096), np.log(4 << 20), size=k)).astype(np.int64) // 256) * 256
    tens = []
    for i in range(k):
        half = rng.random() < 0.5
        t = torch.randn(int(sizes[i]) // (2 if half else 4)).to(torch.float16 if half else torch.float32)
        tens.append(t.pin_memory())
    ok = True
    for t in tens:
        a = attrs(hip, t.data_ptr())
        end = t.data_ptr() + t.numel() * t.element_size()
        if not (a['rc'] == 0 and a['type'] == 1 and a['dev'] == t.data_ptr() and a['range_start'] is not None
                and a['range_start'] <= t.data_ptr() and end <= a['range_start'] + a['range_size']):
            ok = False
            emit({'probe': 'c5_attrs_unexpected', 'attrs': a, 'ptr': t.data_ptr(), 'end': end})
            break
    t0 = time.perf_counter()
    for t in tens:
        attrs(hip, t.data_ptr())
    t1 = time.perf_counter()
    a = PtrAttr()
    for t in tens:
        hip.hipPointerGetAttributes(ctypes.byref(a), ctypes.c_void_p(t.data_ptr()))
    t2 = time.perf_counter()
    emit({'probe': 'attr_query_cost', 'us_per_tensor_3_queries': round((t1 - t0) / k * 1e6, 3),
          'us_per_tensor_attributes_only': round((t2 - t1) / k * 1e6, 3), 'note': 'through ctypes'})
    total = sum(t.numel() * t.element_size() for t in tens)
    if not ok:
        emit({'probe': 'stop', 'reason': 'pinned tensors not mapped at their host address'})
        return
    V = ctypes.c_void_p * k
    ptrs = V(*[t.data_ptr() for t in tens])
    nbytes = (ctypes.c_size_t * k)(*[t.numel() * t.element_size() for t in tens])
    flat = sum((int(b) + 255) // 256 * 256 for b in nbytes)
    fused = torch.empty(flat, dtype=torch.uint8, device=dev)
    ref = [t.clone() for t in tens]
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()

    def timed(fn, reps=3):
        fn()
        torch.cuda.synchronize()
        best = float('inf')
        for _ in range(reps):
            t0 = time.perf_counter()
            fn()
            torch.cuda.synchronize()
            best = min(best, time.perf_counter() - t0)
        return best

    t_pack = timed(lambda: check(lib.ddl_pack(fused.data_ptr(), ptrs, nbytes, k, s1.cuda_stream), 'pack'))
    for t in tens:
        t.zero_()
    t_unpack = timed(lambda: check(lib.ddl_unpack(ptrs, fused.data_ptr(), nbytes, k, s1.cuda_stream), 'unpack'))
    same = all(torch.equal(a, b) for a, b in zip(tens, ref))
    emit({'probe': 'zero_copy_pack_unpack_c5', 'bytes': total, 'pack_ms': round(t_pack * 1e3, 3),
          'pack_GBs': round(total / t_pack / 1e9, 2), 'unpack_ms': round(t_unpack * 1e3, 3),
          'unpack_GBs': round(total / t_unpack / 1e9, 2), 'roundtrip_bit_exact': same})

    # both directions at once: pack into one fused buffer while unpacking another
    fused2 = torch.empty_like(fused)

    def both():
        check(lib.ddl_pack(fused.data_ptr(), ptrs, nbytes, k, s1.cuda_stream), 'pack')
        check(lib.ddl_unpack(ptrs, fused2.data_ptr(), nbytes, k, s2.cuda_stream), 'unpack')
    check(lib.ddl_pack(fused2.data_ptr(), ptrs, nbytes, k, s1.cuda_stream), 'pack')
    t_both = timed(both)
    emit({'probe': 'zero_copy_both_directions_c5', 'bytes_each_way': total, 'ms': round(t_both * 1e3, 3),
          'GBs_each_way': round(total / t_both / 1e9, 2)})

    # DMA per tensor straight from / to the pinned tensors (no host memcpy): one hipMemcpyAsync
    # per bucket, each direction alone and both at once, and mixed with the kernels
    offs, o = [], 0
    for b in nbytes:
        offs.append(o)
        o += (int(b) + 255) // 256 * 256
    base, base2 = fused.data_ptr(), fused2.data_ptr()
    hip.hipMemcpyAsync.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_void_p]
    sh1, sh2 = ctypes.c_void_p(s1.cuda_stream), ctypes.c_void_p(s2.cuda_stream)

    def dma_h2d(dstbase=base):
        for i in range(k):
            hip.hipMemcpyAsync(dstbase + offs[i], ptrs[i], nbytes[i], 1, sh1)

    def dma_d2h(srcbase=base2):
        for i in range(k):
            hip.hipMemcpyAsync(ptrs[i], srcbase + offs[i], nbytes[i], 2, sh2)

    t0 = time.perf_counter()
    dma_h2d()
    t_enq = time.perf_counter() - t0
    torch.cuda.synchronize()
    res = {'probe': 'dma_per_tensor_c5', 'enqueue_us_per_copy': round(t_enq / k * 1e6, 2)}
    for name, fn in (('h2d', dma_h2d), ('d2h', dma_d2h), ('both', lambda: (dma_h2d(), dma_d2h())),
                     ('kernel_h2d_dma_d2h', lambda: (check(lib.ddl_pack(base, ptrs, nbytes, k, s1.cuda_stream), 'p'),
                                                     dma_d2h())),
                     ('dma_h2d_kernel_d2h', lambda: (dma_h2d(), check(lib.ddl_unpack(ptrs, base2, nbytes, k,
                                                                                    s2.cuda_stream), 'u')))):
        t = timed(fn)
        res[name + '_GBs_each_way'] = round(total / t / 1e9, 2)
    emit(res)
    if hasattr(hip, 'hipMemcpyBatchAsync'):
        Vp = ctypes.c_void_p * k
        dsts = Vp(*[base + x for x in offs])
        fail = ctypes.c_size_t()
        hip.hipMemcpyBatchAsync.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t,
                                            ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p,
                                            ctypes.c_void_p]
        rcs = []

        def batch():
            rcs.append(hip.hipMemcpyBatchAsync(dsts, ptrs, nbytes, k, None, None, 0, ctypes.byref(fail), sh1))
        t = timed(batch)
        hip.hipGetLastError()
        emit({'probe': 'hipMemcpyBatchAsync_h2d_c5', 'rc': rcs[-1], 'GBs': round(total / t / 1e9, 2)})

    # DMA reference: one pinned buffer of the same size, H2D, D2H, both at once
    big = torch.empty(total // 4, dtype=torch.float32, pin_memory=True)
    dbig, dbig2 = torch.empty(total // 4, device=dev), torch.empty(total // 4, device=dev)
    big2 = torch.empty_like(big).pin_memory()

    def h2d():
        with torch.cuda.stream(s1):
            dbig.copy_(big, non_blocking=True)

    def d2h():
        with torch.cuda.stream(s2):
            big2.copy_(dbig2, non_blocking=True)

    def dma_both():
        h2d()
        d2h()
    emit({'probe': 'dma_one_pinned_buffer', 'bytes': total, 'h2d_GBs': round(total / timed(h2d) / 1e9, 2),
          'd2h_GBs': round(total / timed(d2h) / 1e9, 2), 'both_GBs_each_way': round(total / timed(dma_both) / 1e9, 2)})

    # hybrids: one direction by the kernel over PCIe, the other by one large DMA of a pinned slot
    def kernel_pack_dma_d2h():
        check(lib.ddl_pack(base, ptrs, nbytes, k, s1.cuda_stream), 'p')
        d2h()

    def dma_h2d_kernel_unpack():
        h2d()
        check(lib.ddl_unpack(ptrs, base2, nbytes, k, s2.cuda_stream), 'u')
    emit({'probe': 'hybrid_c5', 'kernel_pack_with_large_d2h_GBs_each_way': round(total / timed(kernel_pack_dma_d2h) / 1e9, 2),
          'large_h2d_with_kernel_unpack_GBs_each_way': round(total / timed(dma_h2d_kernel_unpack) / 1e9, 2)})


if __name__ == '__main__':
    main()
