"""Host-side half of the engine's test-harness transport (ddl_init_test_transport,
include/ddl_amd_testing.h): the point-to-point groups of every tick move through torch.distributed gloo
on host copies, so several processes can run the whole N>1 engine on one GPU (RCCL refuses two
ranks on one device). Used by tests/_mp_gpu_worker.py and by `bench.py --rehearse` (a
rehearsal of the N>1 bench legs, not a measurement). Never part of the product path."""
import ctypes
import traceback


class P2POp(ctypes.Structure):  # ddl_p2p_op
    _fields_ = [('send', ctypes.c_int), ('peer', ctypes.c_int), ('tag', ctypes.c_int), ('ptr', ctypes.c_void_p),
                ('bytes', ctypes.c_size_t)]


GROUP_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_longlong, ctypes.POINTER(P2POp), ctypes.c_int, ctypes.c_void_p)
MAX_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_longlong, ctypes.POINTER(ctypes.c_float), ctypes.c_int,
                          ctypes.c_void_p)


def _tag(comm_tag, t):
    return int(comm_tag) * 4096 + int(t)  # communicators (world, handler copy) never share a tag


def make_callbacks(dist, torch, rank, world):
    """(group, max) callbacks over the default gloo process group; keep them referenced."""
    def group(comm_tag, ops, count, user):
        try:
            reqs = []
            for i in range(count):
                op = ops[i]
                if op.bytes == 0:
                    continue
                t = torch.frombuffer((ctypes.c_uint8 * op.bytes).from_address(op.ptr), dtype=torch.uint8)
                tg = _tag(comm_tag, op.tag)
                reqs.append(dist.isend(t, op.peer, tag=tg) if op.send else dist.irecv(t, op.peer, tag=tg))
            for r in reqs:
                r.wait()
            return 0
        except Exception:
            traceback.print_exc()
            return 1

    def vmax(comm_tag, vals, count, user):
        try:
            t = torch.tensor([vals[i] for i in range(count)], dtype=torch.float32)
            tg = _tag(comm_tag, 4000)
            if rank == 0:
                for q in range(1, world):
                    o = torch.empty_like(t)
                    dist.recv(o, q, tag=tg)
                    t = torch.maximum(t, o)
                for q in range(1, world):
                    dist.send(t, q, tag=tg + 1)
            else:
                dist.send(t, 0, tag=tg)
                dist.recv(t, 0, tag=tg + 1)
            for i in range(count):
                vals[i] = float(t[i])
            return 0
        except Exception:
            traceback.print_exc()
            return 1

    return GROUP_FN(group), MAX_FN(vmax)


def init_world(lib, dist, torch, rank, world, device=0):
    """ddl_init_test_transport + the token ring, as ddl.torch.communicator.init() does with RCCL.
    Returns the callbacks, which must stay alive as long as the engine."""
    import os
    from ddl.torch.cpp_backend import check
    os.environ['DDL_ALLOW_TEST_TRANSPORT'] = '1'  # the engine refuses the test transport otherwise
    lib.ddl_init_test_transport.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, GROUP_FN, MAX_FN,
                                            ctypes.c_void_p]
    lib.ddl_init_test_transport.restype = ctypes.c_int
    cbs = make_callbacks(dist, torch, rank, world)
    check(lib.ddl_init_test_transport(rank, world, device, cbs[0], cbs[1], None), 'ddl_init_test_transport')
    ep = ctypes.create_string_buffer(256)
    check(lib.ddl_control_listen(ep, 256), 'ddl_control_listen')
    eps = [None] * world
    dist.all_gather_object(eps, ep.value.decode())
    check(lib.ddl_control_connect(';'.join(eps).encode()), 'ddl_control_connect')
    return cbs
