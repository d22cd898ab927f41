"""Keyed host-tensor C5 batch (bench.keyed_host_c5) vs the memcpy workers of the pinned staging
pipeline ("host_copy_threads") and its chunk size (measurement tool, not shipped)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault('ddl_lib', os.path.join(ROOT, 'experiment-distributed-deep-learning_amd', 'lib', 'libddl_amd_testing.so'))  # the testing build (raw kernels, test transport)
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
    # (r03: the copy pool is rebuilt when host_copy_threads changes — r02's sweep ran every
    # setting on the pool built for the first one)
    for pinned in (True, False):
        for threads, chunk in ((0, 32), (3, 32), (7, 32), (11, 32), (15, 32), (15, 16), (15, 64)):
            check(lib.ddl_set_config(b'host_copy_threads', threads), 'cfg')
            check(lib.ddl_set_config(b'host_chunk_bytes', chunk << 20), 'cfg')
            r = bench.keyed_host_c5(lib, comm, steps=3, pinned=pinned)
            print(json.dumps({'pinned': pinned, 'host_copy_threads': threads, 'chunk_MiB': chunk, 'ms': r['ms'],
                              'GiBs': r['bucket_GiBs'], 'engine_thread': r['engine_thread']}), flush=True)


if __name__ == '__main__':
    main()
