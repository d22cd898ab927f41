"""C4 fp16 fold (2 MiB chunk, P = 8) in the tile vs the run form, bench.fold_roofline timing (measurement)."""
import sys, os, json
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault('ddl_lib', os.path.join(ROOT, 'experiment-distributed-deep-learning_amd', 'lib', 'libddl_amd_testing.so'))  # the testing build (raw kernels, test transport)
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, 'experiment-distributed-deep-learning_amd'))
import torch, bench
from ddl.torch.cpp_backend import CPPBackend
lib = CPPBackend.c_api()
dev = torch.device('cuda', 0); torch.cuda.set_device(dev)
sh = torch.cuda.current_stream().cuda_stream
for rep in range(3):
    for form in (1, 2):
        r = bench.fold_roofline(lib, dev, sh, 16 << 20, half=True, form=form)
        print(json.dumps({'form': form, 'us': r['us'], 'frac': r['frac_of_peak']}), flush=True)
