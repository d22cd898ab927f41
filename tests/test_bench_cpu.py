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
