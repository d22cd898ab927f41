"""bench.py's N>1 watchdog: a leg that hangs must end the run with a non-zero
exit code, and rank 0's line must still be printed, carrying `incomplete`. The run goes through
bench.py's own launcher (`--gpus 2`: spawn_ranks) with the watchdog self-test hook, which stalls
one rank in a gloo barrier after rank 0 holds a line — no GPU needed."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_hung_leg_exits_nonzero_with_incomplete_line():
    env = dict(os.environ, DDL_BENCH_WATCHDOG_SELFTEST='1')
    env.pop('WORLD_SIZE', None)
    p = subprocess.run([sys.executable, os.path.join(ROOT, 'bench.py'), '--gpus', '2', '--watchdog-s', '4'],
                       env=env, capture_output=True, text=True, timeout=180)
    assert p.returncode == 3, (p.returncode, p.stderr[-2000:])
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith('{')]
    assert len(lines) == 1, p.stdout
    line = json.loads(lines[0])
    assert line['selftest'] is True
    assert 'selftest_hang' in line['incomplete'], line


def _bench():
    import importlib.util
    spec = importlib.util.spec_from_file_location('bench_mod', os.path.join(ROOT, 'bench.py'))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def test_lane_split_fields():
    """The unpack lane's per-step split in every host leg's engine_thread."""
    b = _bench()
    d = b.lane_split(18.2, 54.05, 2446361088, 74)
    assert d['lane_d2h_wait_ms'] == 18.2 and d['lane_copy_ms'] == 54.05 and d['lane_jobs'] == 74
    assert d['lane_copy_GBs'] == round(2446361088 / 0.05405 / 1e9, 2)
    assert b.lane_split(0.0, 0.0, 0, 0)['lane_copy_GBs'] is None  # pinned legs: no staged unpack


def test_tuner_table_shape():
    import ctypes
    b = _bench()
    cfgs = (ctypes.c_longlong * 128)(*([1, 1, 256 << 10, 16] + [4, 1, 2 << 20, 8]))
    tms = (ctypes.c_float * 32)(0.5, 0.25)
    t = b.tuner_table(ctypes.c_int(1), ctypes.c_int(2), cfgs, tms)
    assert t['chosen'] == {'algo': 'direct_gather', 'rings': 1, 'slice_KiB': 2048, 'max_slices': 8, 'ms': 0.25}
    assert [c['slice_KiB'] for c in t['candidates']] == [256, 2048]
