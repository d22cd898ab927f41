#!/bin/bash
# r02 s5: N=2 / N=4 rehearsals of the N>1 bench on one GPU (every leg, incl. keyed_c1_latency).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=${O:-gpurun_out/s5c}; mkdir -p $O
for N in 2 4; do
  timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node $N --master-addr 127.0.0.1 \
    --master-port $((29575 + N)) bench.py --gpus $N --steps 5 --warmup 2 --bucket-mib 8 --size-sweep-max-mib 16 \
    --rehearse > $O/rehearse$N.json 2> $O/rehearse$N.err
  rc=$?; echo "rehearse N=$N rc=$rc"; python -c "
import json,sys;d=json.loads(open('$O/rehearse$N.json').read().strip().splitlines()[-1])
print({k:d.get(k) for k in ('value','unit','leg_errors','keyed_c1_latency','keyed_bucket_stream')})
print('parity', d.get('parity_vs_mpich_order', {}).get('bit_exact'))"
  [ $rc -eq 0 ] || exit $rc
done
