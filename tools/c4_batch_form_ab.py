"""C4's batched fp16 fold (8 buckets' 2 MiB chunks per launch, P = 8) in the tile vs the run form,
interleaved rounds, bench.fold_batch_roofline timing (measurement)."""
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
for rep in range(3):
    for per_launch in (8,):
        for form in (1, 2):
            r = bench.fold_batch_roofline(lib, dev, sh, per_launch=per_launch, form=form)
            print(json.dumps({'rep': rep, 'form': form, 'per_launch': per_launch, 'us': r['us'],
                              'frac': r['frac_of_peak']}), flush=True)
            torch.cuda.empty_cache()
