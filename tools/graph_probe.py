"""Which part of the engine survives hipGraph capture (diagnostic, one mode per process):
  local   — P virtual ranks, D2D copies for the moves (multi-stream fork / join only)
  gather  — one ncclAllGather on a one-rank RCCL communicator
  group   — one RCCL group of self send / recv pairs (the loopback's moves)
  loop    — the RCCL loopback allreduce (what tests/test_graph_gpu.py captures)
  fold    — one N-input fold kernel launch (single stream)
  ring2   — local world P = 2, ring schedule (two-input reduce kernels, no fold)
  rawlocal— `local` captured with hipStreamBeginCapture through ctypes (no torch graph)
    python graph_probe.py <mode> [algo] [capture_mode: 0 = posted serially (default), 2 = as a
    single-stream DAG; r03's forked mode 1 was removed in r04]
Prints one line per stage; a crash names the last stage reached."""
import ctypes
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault('ddl_lib', os.path.join(ROOT, 'experiment-distributed-deep-learning_amd', 'lib', 'libddl_amd_testing.so'))  # the testing build (raw kernels, test transport)
sys.path.insert(0, os.path.join(ROOT, 'experiment-distributed-deep-learning_amd'))
from ddl.torch.cpp_backend import CPPBackend  # noqa: E402


def say(*a):
    print(*a, flush=True)


def main(mode, P=3, n=300, algo=1, capture_mode=0):
    lib = CPPBackend.c_api()
    dev = torch.device('cuda', 0)
    torch.cuda.set_device(dev)
    lib.ddl_set_config(b'capture_mode', capture_mode)
    lib.ddl_set_config(b'tune', 0)
    lib.ddl_set_config(b'algo', algo)
    lib.ddl_set_config(b'slice_bytes', 64 << 10)
    s = torch.cuda.Stream()
    ins = [torch.randn(n, device=dev) for _ in range(P)]
    outs = [torch.empty_like(t) for t in ins]
    send = (ctypes.c_void_p * P)(*[t.data_ptr() for t in ins])
    recv = (ctypes.c_void_p * P)(*[t.data_ptr() for t in outs])
    if mode in ('gather', 'group', 'loop'):
        assert lib.ddl_rccl_loopback_init(0) == 0, lib.ddl_last_error()
        say('loopback init ok')
    if mode == 'ring2':
        lib.ddl_set_config(b'reference_order', 0)
        lib.ddl_set_config(b'algo', 0)
    if mode == 'rawlocal':
        return raw_capture(lib, s, P, send, recv, n, outs)

    def call():
        if mode in ('local', 'ring2'):
            Q = 2 if mode == 'ring2' else P
            return lib.ddl_local_ring_allreduce(Q, send, recv, n, 1, 0, s.cuda_stream)
        if mode == 'fold':
            return lib.ddl_reduce_fold(ctypes.c_void_p(outs[0].data_ptr()), ctypes.c_void_p(ins[0].data_ptr()),
                                       (ctypes.c_void_p * 2)(ins[1].data_ptr(), ins[2].data_ptr()), 2, n, 1,
                                       s.cuda_stream)
        if mode == 'gather':
            return lib.ddl_rccl_loopback_allgather(ctypes.c_void_p(ins[0].data_ptr()),
                                                   ctypes.c_void_p(outs[0].data_ptr()), n * 4, s.cuda_stream)
        if mode == 'group':
            return lib.ddl_rccl_loopback_allreduce(P, send, recv, n, 1, s.cuda_stream)
        return lib.ddl_rccl_loopback_allreduce(P, send, recv, n, 1, s.cuda_stream)

    with torch.cuda.stream(s):
        assert call() == 0, lib.ddl_last_error()
    torch.cuda.synchronize()
    say(mode, 'eager ok')
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        st = call()
        say(mode, 'captured call status', st, lib.ddl_last_error() if st else '')
    say(mode, 'capture ended')
    want = [o.clone() for o in outs]
    for o in outs:
        o.zero_()
    g.replay()
    torch.cuda.synchronize()
    say(mode, 'replay ok', all(torch.equal(a, b) for a, b in zip(outs, want)))
    del g
    if mode in ('gather', 'group', 'loop'):
        assert lib.ddl_rccl_loopback_finalize() == 0


def hip_runtime():
    """The HIP runtime torch and the engine already share, matched by soname with RTLD_NOLOAD.
    (r02's probe loaded 'libamdhip64.so' by file name: /opt/rocm's copy, a SECOND runtime beside
    torch's bundled one, handed torch's stream to it — the `rawlocal` segfault.)"""
    vp, ci = ctypes.c_void_p, ctypes.c_int
    hip = ctypes.CDLL('libamdhip64.so.7', mode=os.RTLD_NOLOAD | os.RTLD_NOW)
    for name, res, args in (('hipStreamBeginCapture', ci, [vp, ci]),
                            ('hipStreamEndCapture', ci, [vp, ctypes.POINTER(vp)]),
                            ('hipGraphGetNodes', ci, [vp, vp, ctypes.POINTER(ctypes.c_size_t)]),
                            ('hipGraphInstantiate', ci, [ctypes.POINTER(vp), vp, vp, vp, ctypes.c_size_t]),
                            ('hipGraphLaunch', ci, [vp, vp])):
        f = getattr(hip, name)
        f.restype, f.argtypes = res, args
    return hip


def raw_capture(lib, s, P, send, recv, n, outs):
    hip = hip_runtime()
    vp = ctypes.c_void_p
    st = ctypes.c_void_p(s.cuda_stream)
    assert lib.ddl_local_ring_allreduce(P, send, recv, n, 1, 0, s.cuda_stream) == 0
    torch.cuda.synchronize()
    say('rawlocal eager ok')
    assert hip.hipStreamBeginCapture(st, 0) == 0  # hipStreamCaptureModeGlobal
    rc = lib.ddl_local_ring_allreduce(P, send, recv, n, 1, 0, s.cuda_stream)
    say('rawlocal captured call status', rc)
    g = vp()
    rc = hip.hipStreamEndCapture(st, ctypes.byref(g))
    say('rawlocal end capture rc', rc)
    nn = ctypes.c_size_t(0)
    hip.hipGraphGetNodes(g, None, ctypes.byref(nn))
    say('rawlocal nodes', nn.value)
    x = vp()
    rc = hip.hipGraphInstantiate(ctypes.byref(x), g, None, None, ctypes.c_size_t(0))
    say('rawlocal instantiate rc', rc)
    want = [o.clone() for o in outs]
    for o in outs:
        o.zero_()
    torch.cuda.synchronize()
    rc = hip.hipGraphLaunch(x, st)
    torch.cuda.synchronize()
    say('rawlocal replay rc', rc, all(torch.equal(a, b) for a, b in zip(outs, want)))


if __name__ == '__main__':
    m = sys.argv[1]
    algo = int(sys.argv[2]) if len(sys.argv) > 2 else 1
    capture_mode = int(sys.argv[3]) if len(sys.argv) > 3 else 0
    if m == 'group':  # the one-shot schedule: one group of self pairs, one fold
        algo = 2
    main(m, algo=algo, capture_mode=capture_mode)
