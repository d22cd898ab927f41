"""A/B of the fold's cache policy (the policy is chosen from the batch's summed
elements, so 8 C4 chunks of 2 MiB = 16 MiB take non-temporal loads, where the per-chunk rule
would read them through the caches). With `--single`, also single-chunk launches (one problem per
launch) at 2 MiB fp16 and 4 / 8 MiB fp32, P = 8: the sizes the per-chunk rule reads through the
caches.

C4's folds as the grouped allreduce launches them: 8 problems per launch (FoldBatch), each a
2 MiB fp16 chunk with 7 received inputs (k_sumN_tile<DDL_HALF, 7>), policy forced through
ddl_testing_fold_variant: 4 = plain loads + write-through store, 5 = non-temporal loads +
write-through store. Two residencies:
  * hbm: 64 buckets' operands (1.2 GB) rotate launch by launch, 8 launches per pass;
  * cache: the 8 buckets of ONE launch (151 MB, inside the 256 MiB Infinity Cache), relaunched —
    the grouped allreduce's tick, whose received slices RCCL has just written.
Each measurement is a hipGraph of the pass replayed between HIP events; the two policies are
interleaved, 3 rounds. One JSON line."""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'experiment-distributed-deep-learning_amd'))
os.environ.setdefault('ddl_lib', os.path.join(ROOT, 'experiment-distributed-deep-learning_amd', 'lib',
                                              'libddl_amd_testing.so'))

import torch  # noqa: E402

from ddl.torch.cpp_backend import CPPBackend, check  # noqa: E402

NB, DT_HALF, PER = 7, 19, 8


def measure(lib, dev, per, chunk_bytes, half, cases):
    """{residency: {variant: [us per launch] x 3 rounds}} for folds of `per` problems per launch."""
    es = 2 if half else 4
    n = chunk_bytes // es
    V = ctypes.c_void_p
    dt = DT_HALF if half else 1

    def pass_graph(buckets):
        sets = [[torch.rand(n, device=dev).to(torch.float16 if half else torch.float32) for _ in range(NB + 2)]
                for _ in range(buckets)]
        launches = []
        for k in range(0, buckets, per):
            grp = sets[k:k + per]
            launches.append(((V * per)(*[b[-1].data_ptr() for b in grp]), (V * per)(*[b[0].data_ptr() for b in grp]),
                             (V * (per * NB))(*[t.data_ptr() for b in grp for t in b[1:-1]]),
                             (ctypes.c_size_t * per)(*[n] * per)))
        reps = max(1, 8 // len(launches))  # the cache case relaunches its one problem set

        def run(stream):
            for _ in range(reps):
                for outs, as_, ins, ns in launches:
                    check(lib.ddl_reduce_fold_batch(per, outs, as_, ins, NB, ns, dt, 0, stream),
                          'ddl_reduce_fold_batch')
        return sets, run, len(launches) * reps

    res = {'problems_per_launch': per, 'chunk_bytes': chunk_bytes, 'dtype': 'fp16' if half else 'fp32',
           'algorithmic_bytes_per_launch': per * (NB + 2) * chunk_bytes}
    for residency, buckets in cases:
        sets, run, launches = pass_graph(buckets)
        graphs = {}
        for v in (4, 5):
            check(lib.ddl_testing_fold_variant(v), 'ddl_testing_fold_variant')
            try:
                run(torch.cuda.current_stream().cuda_stream)
                torch.cuda.synchronize()
                gs = torch.cuda.Stream()
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g, stream=gs):  # the policy is fixed at capture
                    run(gs.cuda_stream)
                graphs[v] = (g, gs)
            finally:
                check(lib.ddl_testing_fold_variant(-1), 'ddl_testing_fold_variant')
        times = {4: [], 5: []}
        for _ in range(3):
            for v in (4, 5):
                g, gs = graphs[v]
                with torch.cuda.stream(gs):
                    g.replay()
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record(gs)
                    g.replay()
                    e1.record(gs)
                torch.cuda.synchronize()
                times[v].append(round(e0.elapsed_time(e1) * 1e3 / launches, 2))
        res[residency] = {f'variant{v}_us_per_launch': t for v, t in times.items()}
        res[residency].update({f'variant{v}_TBs_best': round(res['algorithmic_bytes_per_launch'] / min(t) / 1e6, 3)
                               for v, t in times.items()})
        res[residency]['operand_bytes'] = buckets * (NB + 2) * chunk_bytes
        del graphs, sets
    return res


def main():
    lib = CPPBackend.c_api()
    dev = torch.device('cuda', 0)
    torch.cuda.set_device(dev)
    out = {'batch8_fp16_2MiB': measure(lib, dev, PER, 2 << 20, True, (('hbm', 64), ('cache', 8)))}
    if '--single' in sys.argv:
        # single-chunk launches: HBM = enough rotating sets to exceed the 256 MiB Infinity Cache
        out['single_fp16_2MiB'] = measure(lib, dev, 1, 2 << 20, True, (('hbm', 32), ('cache', 1)))
        out['single_fp32_4MiB'] = measure(lib, dev, 1, 4 << 20, False, (('hbm', 16), ('cache', 1)))
        out['single_fp32_8MiB'] = measure(lib, dev, 1, 8 << 20, False, (('hbm', 8), ('cache', 1)))
    for a in sys.argv[1:]:
        if a.startswith('--fp32-mib='):  # more single fp32 chunk sizes (the rule's boundary)
            for mib in (float(x) for x in a.split('=', 1)[1].split(',')):
                b = int(mib * (1 << 20)) // 256 * 256
                out[f'single_fp32_{mib:g}MiB'] = measure(lib, dev, 1, b, False, (('hbm', max(2, (600 << 20) // (9 * b))),
                                                                             ('cache', 1)))
    print(json.dumps(out), flush=True)


if __name__ == '__main__':
    main()
