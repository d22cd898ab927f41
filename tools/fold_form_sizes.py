"""The P = 8 fp32 fold in the tile vs the run form at chunk sizes around the 8 MiB switch
(bench.fold_roofline timing: 2 rotating sets, 20 launches per graph; measurement)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault('ddl_lib', os.path.join(ROOT, 'experiment-distributed-deep-learning_amd', 'lib', 'libddl_amd_testing.so'))  # the testing build (raw kernels, test transport)
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'experiment-distributed-deep-learning_amd'))
import torch  # noqa: E402

import bench  # noqa: E402
from ddl.torch.cpp_backend import CPPBackend  # noqa: E402

lib = CPPBackend.c_api()
dev = torch.device('cuda', 0)
torch.cuda.set_device(dev)
sh = torch.cuda.current_stream().cuda_stream
bench.fold_roofline(lib, dev, sh, 16 << 20, form=1)  # warm the process's first graph
for rep in range(2):
    for chunk_mib in (2, 4, 8, 16, 32):
        for form in (1, 2):
            r = bench.fold_roofline(lib, dev, sh, (chunk_mib << 20) * 8, order=1, form=form)
            print(json.dumps({'chunk_MiB': chunk_mib, 'form': ('tile', 'run')[form - 1], 'us': r['us'],
                              'TBps': round(r['achieved_GBs'] / 1e3, 3)}), flush=True)
