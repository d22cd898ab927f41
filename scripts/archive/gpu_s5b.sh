#!/bin/bash
# r02 s5: pipelined keyed rounds at one rank (probe), DP overlap probe, N=2 / N=4 rehearsals of
# the N>1 bench (every leg, incl. keyed_bucket_stream). Stops at the first failing step.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/s5b; mkdir -p $O
timeout -k 10 300 python -u tools/round_pipeline_probe.py > $O/round_pipeline.jsonl 2> $O/round_pipeline.err
rc=$?; echo "round_pipeline rc=$rc"; cat $O/round_pipeline.jsonl; tail -3 $O/round_pipeline.err; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/dp_overlap_probe.py > $O/dp_overlap.json 2> $O/dp_overlap.err
rc=$?; echo "dp_overlap rc=$rc"; cat $O/dp_overlap.json; [ $rc -eq 0 ] || exit $rc
for N in 2 4; do
  timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node $N --master-addr 127.0.0.1 \
    --master-port $((29555 + N)) bench.py --gpus $N --steps 5 --warmup 2 --bucket-mib 8 --size-sweep-max-mib 16 \
    --rehearse > $O/rehearse$N.json 2> $O/rehearse$N.err
  rc=$?; echo "rehearse N=$N rc=$rc"; python -c "
import json,sys;d=json.loads(open('$O/rehearse$N.json').read().strip().splitlines()[-1])
print({k:d.get(k) for k in ('value','unit','check','leg_errors','keyed_bucket_stream')})
print('parity', d.get('parity_vs_mpich_order', {}).get('bit_exact'))"
  [ $rc -eq 0 ] || exit $rc
done
