#!/bin/bash
# product reduce kernel with the per-size cache policy: parity tests, then the N=1 sweep under the
# new default and under the r02 policies forced (0 = plain, 7 = all nt), interleaved, same box
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r02l; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_reduce_gpu.py -x -q --timeout 120 --timeout-method thread > $O/pytest_reduce.log 2>&1
rc=$?; echo "pytest reduce rc=$rc"; tail -3 $O/pytest_reduce.log; [ $rc -eq 0 ] || exit $rc
for R in 1 2; do
  for V in default 7 0; do
    if [ $V = default ]; then E=""; else E="DDL_REDUCE_VARIANT=$V"; fi
    env $E timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-host --no-fusion --no-cpu-baseline $([ $V = default ] && [ $R = 1 ] || echo --no-variants) > $O/bench_${V}_$R.json 2> $O/bench_${V}_$R.err
    rc=$?; echo "bench $V round $R rc=$rc"; [ $rc -eq 0 ] || { tail -5 $O/bench_${V}_$R.err; exit $rc; }
  done
done
python3 - <<'PY'
import json
O='gpurun_out/r02l'
rows={}
for V in ['default','7','0']:
    for R in (1,2):
        d=json.load(open(f'{O}/bench_{V}_{R}.json'))
        for p in d['sweep_fp32']:
            rows.setdefault(p['bytes'],{}).setdefault(V,[]).append(p['hbm_GBs'])
print('bytes default(new) nt_all(7) plain(0)  [best of 2, HBM GB/s]')
for b in sorted(rows):
    print(b, *[max(rows[b][v]) for v in ['default','7','0']])
d=json.load(open(f'{O}/bench_default_1.json'))
print('headline', d['value'], d['roofline'], d.get('variants_achieved_GBs'))
PY
