"""Why the C4 single-chunk fold reads 3.3 us in the bench's graph replay and 4.4-4.5 us in
rocprofv3's per-dispatch average.

The same kernel (k_sumN_tile<DDL_HALF, 7>, one fp16 chunk of about 2 MiB, 7 received inputs) is
launched four ways in one process. Each way uses a chunk a few 2 KiB tiles shorter than 2 MiB, so
its grid differs and rocprofv3's trace splits the ways by (kernel, grid):

  grid 1021  isolated:      launch, then synchronise the stream (nothing queued behind it)
  grid 1020  eager burst:   200 launches from Python back to back
  grid 1019  graph replay:  20 launches captured into a hipGraph, replayed
  grid 1018  isolated, HBM: as 1021, with 24 rotating operand sets (432 MiB, beyond the
                            Infinity Cache) instead of 2 (36 MiB, cache-resident)

HIP events time each way on the launch stream. Run under
  rocprofv3 --kernel-trace --stats -d <dir> -- python3 tools/c4_dispatch_probe.py
and summarize with scripts/prof_summarize.py <dir>: the per-grid averages next to this script's
JSON line say which clock reads what.
"""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'experiment-distributed-deep-learning_amd'))
_TESTING = os.path.join(ROOT, 'experiment-distributed-deep-learning_amd', 'lib', 'libddl_amd_testing.so')
if os.path.exists(_TESTING):  # the raw-kernel entry points live in the testing library
    os.environ.setdefault('ddl_lib', _TESTING)

import torch  # noqa: E402

from ddl.torch.cpp_backend import CPPBackend, check  # noqa: E402

NB, DT_HALF = 7, 19


def main():
    lib = CPPBackend.c_api()
    dev = torch.device('cuda', 0)
    torch.cuda.set_device(dev)
    stream = torch.cuda.current_stream(dev)
    sh = stream.cuda_stream
    P = ctypes.c_void_p * NB

    def sets_for(tiles_short, nsets):
        n = ((2 << 20) - 2048 * tiles_short) // 2
        return n, [[torch.rand(n, device=dev).half() for _ in range(NB + 2)] for _ in range(nsets)]

    def launch(n, b, s):
        check(lib.ddl_reduce_fold_ordered(b[-1].data_ptr(), b[0].data_ptr(), P(*[t.data_ptr() for t in b[1:-1]]),
                                          NB, n, DT_HALF, 0, s), 'ddl_reduce_fold_ordered')

    out = {}

    def isolated(tag, tiles_short, nsets, reps=60):
        n, sets = sets_for(tiles_short, nsets)
        ts = []
        for k in range(reps + 5):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            launch(n, sets[k % nsets], sh)
            e1.record(stream)
            torch.cuda.synchronize()
            if k >= 5:
                ts.append(e0.elapsed_time(e1) * 1e3)
        ts.sort()
        out[tag] = {'grid': (n * 2 // 16 + 128) // 128, 'operand_sets': nsets, 'events_us_median': round(ts[len(ts) // 2], 2),
                    'events_us_min': round(ts[0], 2), 'launches': reps + 5}

    isolated('isolated_cache', 4, 2)
    # eager burst
    n, sets = sets_for(5, 2)
    for k in range(10):
        launch(n, sets[k % 2], sh)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for k in range(200):
        launch(n, sets[k % 2], sh)
    e1.record(stream)
    torch.cuda.synchronize()
    out['eager_burst_cache'] = {'grid': (n * 2 // 16 + 128) // 128, 'operand_sets': 2,
                                'events_us_per_launch': round(e0.elapsed_time(e1) * 1e3 / 200, 2), 'launches': 210}
    # graph replay
    n, sets = sets_for(6, 2)
    launch(n, sets[0], sh)
    torch.cuda.synchronize()
    gs = torch.cuda.Stream()
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph, stream=gs):
        for k in range(20):
            launch(n, sets[k % 2], gs.cuda_stream)
    rounds = []
    for _ in range(10):
        with torch.cuda.stream(gs):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(gs)
            graph.replay()
            e1.record(gs)
        torch.cuda.synchronize()
        rounds.append(e0.elapsed_time(e1) * 1e3 / 20)
    out['graph_replay_cache'] = {'grid': (n * 2 // 16 + 128) // 128, 'operand_sets': 2,
                                 'events_us_per_launch_rounds': [round(r, 2) for r in rounds],
                                 'events_us_per_launch_mean': round(sum(rounds) / len(rounds), 2),
                                 'launches': 1 + 200}
    del graph
    isolated('isolated_hbm', 7, 24)
    out['algorithmic_bytes_per_launch_2MiB'] = 9 * (2 << 20)
    print(json.dumps(out), flush=True)


if __name__ == '__main__':
    main()
