"""Quarter chunks at the ends of host-staged transfers ("host_taper" 0 / 1 / 2) vs chunk size,
interleaved in one process (measurement tool, not shipped): ddl_allreduce_host on a 256 MiB
pinned bucket (bench.host_resident_rate) and the keyed C5 batch of pinned / pageable tensors
(bench.keyed_host_c5).

    python tools/host_taper_ab.py > gpurun_out/host_taper_ab.jsonl"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'experiment-distributed-deep-learning_amd'))


def main():
    import torch
    import bench
    from ddl.torch.communicator import Communicator
    from ddl.torch.cpp_backend import CPPBackend, check
    torch.cuda.set_device(0)
    lib = CPPBackend.c_api()
    comm = Communicator.world()
    for rep in range(3):
        for taper in (2, 1, 0):
            check(lib.ddl_set_config(b'host_taper', taper), 'cfg')
            for chunk in (16, 32, 64):
                check(lib.ddl_set_config(b'host_chunk_bytes', chunk << 20), 'cfg')
                r = bench.host_resident_rate(lib, comm, 256 << 20, reps=8)
                print(json.dumps({'rep': rep, 'leg': 'host_resident', 'host_taper': taper, 'chunk_MiB': chunk,
                                  'ms': r['ms'], 'GiBs': r['bucket_GiBs']}), flush=True)
            check(lib.ddl_set_config(b'host_chunk_bytes', 32 << 20), 'cfg')
            for pinned in (True, False):
                r = bench.keyed_host_c5(lib, comm, steps=3, pinned=pinned)
                print(json.dumps({'rep': rep, 'leg': 'keyed_host_c5' + ('_pinned' if pinned else ''),
                                  'host_taper': taper, 'chunk_MiB': 32, 'ms': r['ms'],
                                  'engine_thread': r['engine_thread']}), flush=True)
    check(lib.ddl_set_config(b'host_taper', 0), 'cfg')


if __name__ == '__main__':
    main()
