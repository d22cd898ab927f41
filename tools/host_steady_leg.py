"""The bench's pageable host C5 leg alone (bench.keyed_host_c5_steady): 10 consecutive 4096-tensor
batches per way, median / p90 / last. For A/Bs of the torch mirror's per-batch cost (measurement)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402  (sets ddl_lib to the testing build)

import torch  # noqa: E402

from ddl.torch.communicator import Communicator  # noqa: E402

torch.cuda.set_device(0)
res = bench.keyed_host_c5_steady(Communicator.world())
print(json.dumps({k: ({kk: vv for kk, vv in v.items() if kk != 'step_ms'} if isinstance(v, dict) else v)
                  for k, v in res.items()}), flush=True)
