"""Pack/unpack kernel variants on the C5 bucket set (run on the GPU box): DDL_PACK_VARIANT 1, 2,
3 = segment tiles of 1 KiB (64 lanes, default), 2 KiB (128 lanes), 4 KiB (128 lanes x 2).
`python tools/pack_tune.py child` runs the current variant once (e.g. under rocprofv3 --pmc)."""
import ctypes
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

if len(sys.argv) == 1:
    for v in [int(x) for x in os.environ.get('VARIANTS', '1 2 3').split()]:
        env = dict(os.environ, DDL_PACK_VARIANT=str(v))
        out = subprocess.run([sys.executable, __file__, 'child'], env=env, capture_output=True, text=True, timeout=300)
        print(f'variant {v}: {out.stdout.strip()} {out.stderr.strip()[-300:] if out.returncode else ""}', flush=True)
    sys.exit(0)

sys.path.insert(0, os.path.join(ROOT, 'experiment-distributed-deep-learning_amd'))
import numpy as np  # noqa: E402
import torch  # noqa: E402
from ddl.torch.cpp_backend import CPPBackend  # noqa: E402

lib = CPPBackend.c_api()
rng = np.random.default_rng(5)
k = 4096
sizes = (np.exp(rng.uniform(np.log(4096), np.log(4 << 20), size=k)).astype(np.int64) // 256) * 256
ts = [torch.empty(int(s), dtype=torch.uint8, device='cuda') for s in sizes]
total = sum(int(s) for s in sizes)
fused = torch.empty(total + 256 * k, dtype=torch.uint8, device='cuda')
V = ctypes.c_void_p * k
ptrs = V(*[t.data_ptr() for t in ts])
nb = (ctypes.c_size_t * k)(*[int(s) for s in sizes])
sh = torch.cuda.current_stream().cuda_stream
for _ in range(3):
    lib.ddl_pack(fused.data_ptr(), ptrs, nb, k, sh)
    lib.ddl_unpack(ptrs, fused.data_ptr(), nb, k, sh)
best = {}
for d in ('pack', 'unpack'):
    ts_ = []
    for _ in range(5):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(4):
            if d == 'pack':
                lib.ddl_pack(fused.data_ptr(), ptrs, nb, k, sh)
            else:
                lib.ddl_unpack(ptrs, fused.data_ptr(), nb, k, sh)
        e1.record()
        torch.cuda.synchronize()
        ts_.append(e0.elapsed_time(e1) / 4)
    best[d] = min(ts_)
print(' '.join(f'{d} {t * 1e3:.0f} us {2 * total / (t / 1e3) / 1e12:.2f} TB/s' for d, t in best.items()))
