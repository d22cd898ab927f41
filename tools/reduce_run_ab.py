"""A/B of the two-input reduce's forms (r05): the shipped tile form (one 2 KiB tile per 128-lane
workgroup, both operands' loads in flight together) against the run form (variant bit 32: a
workgroup owns an 8-tile run and streams a's run, then b's; bit 64: 4-tile runs), each with the
cache bits default_variant picks at that size, acc += in over fp32 buckets of 16 MiB - 1 GiB,
3 rotating buffer sets (beyond the Infinity Cache from 64 MiB), interleaved rounds, HIP events on
the launch stream. One JSON line: TB/s per (size, form), best of the rounds."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'experiment-distributed-deep-learning_amd'))
os.environ.setdefault('ddl_lib', os.path.join(ROOT, 'experiment-distributed-deep-learning_amd', 'lib',
                                              'libddl_amd_testing.so'))

import torch  # noqa: E402

from ddl.torch.cpp_backend import CPPBackend, check  # noqa: E402


def policy(nbytes):  # the cache bits of reduce_kernels.hip default_variant (kReduceBands), form aside
    if nbytes >= 256 << 20:
        return 7
    if nbytes < 12 << 20 or (22 << 20) <= nbytes < (42 << 20):
        return 16
    return 19


def main():
    lib = CPPBackend.c_api()
    dev = torch.device('cuda', 0)
    torch.cuda.set_device(dev)
    s = torch.cuda.current_stream(dev)
    sizes = [int(x) << 20 for x in (sys.argv[1] if len(sys.argv) > 1 else '16,64,256,1024').split(',')]
    out = {}
    for size in sizes:
        n = size // 4
        sets = [(torch.rand(n, device=dev), torch.rand(n, device=dev)) for _ in range(3)]
        pol = policy(size)
        forms = {'tile': pol, 'run8': 32 | pol, 'run4': 96 | pol}
        if len(sys.argv) > 2:  # explicit forms: name:variant,... (e.g. tile19:19,run4_19:115)
            forms = {k: int(v) for k, v in (f.split(':') for f in sys.argv[2].split(','))}
        reps = max(6, min(60, (3 << 30) // size))
        best = {k: float('inf') for k in forms}
        cnt = [0]

        def launch(v):
            a, b = sets[cnt[0] % 3]
            cnt[0] += 1
            check(lib.ddl_reduce_sum2_variant(v, a.data_ptr(), a.data_ptr(), b.data_ptr(), n, 1, s.cuda_stream),
                  'ddl_reduce_sum2_variant')
        for k, v in forms.items():
            for _ in range(3):
                launch(v)
        torch.cuda.synchronize()
        for _ in range(4):
            for k, v in forms.items():
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(s)
                for _ in range(reps):
                    launch(v)
                e1.record(s)
                torch.cuda.synchronize()
                best[k] = min(best[k], e0.elapsed_time(e1) / reps)
        out[f'{size >> 20}MiB'] = {k: round(3 * size / (t / 1e3) / 1e12, 3) for k, t in best.items()}
        out[f'{size >> 20}MiB']['cache_bits'] = pol
        del sets
    print(json.dumps(out), flush=True)


if __name__ == '__main__':
    main()
