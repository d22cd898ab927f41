"""No device-synchronising call on the product's data paths (r06). hipFree /
hipHostFree / hipDeviceSynchronize wait for every stream of the device; on a thread that posts
RCCL work while another communicator's RCCL kernels are in flight, that deadlocked a 5-rank RCCL
world (profiles/r06/s6) — outgrown buffers are retired instead (common.h retire_device). This
check reads the product sources: such calls may appear only in destructors and in free_retired()
(ddl_finalize), never in a function that runs while collectives are in flight. The test harness
(test_worlds.cpp, c_api_testing.cpp) is not the product and is not checked."""
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, 'experiment-distributed-deep-learning_amd', 'csrc')
HARNESS = {'test_worlds.cpp', 'c_api_testing.cpp', 'deptrace.cpp'}
SYNCING = re.compile(r'\b(hipFree|hipHostFree|hipDeviceSynchronize)\s*\(')
DEFINITION = re.compile(r'^[A-Za-z_][\w:<>,\s\*&~]*\([^;]*$')  # a function definition's first line, column 0
ALLOWED = ('~', 'free_retired')


def _enclosing(lines, i):
    for j in range(i, -1, -1):
        ln = lines[j]
        if ln and not ln[0].isspace() and ln[0] not in '}#/' and DEFINITION.match(ln):
            return ln.strip()
    return ''


def test_device_synchronising_calls_only_in_teardown():
    offenders = []
    for f in sorted(os.listdir(CSRC)):
        if not f.endswith(('.cpp', '.hip', '.h')) or f in HARNESS:
            continue
        lines = open(os.path.join(CSRC, f)).read().splitlines()
        for i, ln in enumerate(lines):
            code = ln.split('//')[0]
            if SYNCING.search(code):
                fn = _enclosing(lines, i)
                if not any(a in fn for a in ALLOWED):
                    offenders.append(f'{f}:{i + 1} in {fn!r}')
    assert not offenders, offenders
