"""Loader of the native engine (mirror of reference src/py/ddl/tensorflow/cpp_backend.py:16-80).

The reference loads one library twice — as a TF op library and through ctypes. Here there is
no op library: every call goes through the C-ABI of lib/libddl_amd.so (include/ddl_amd.h).
`import torch` happens first so the engine binds to the HIP runtime (and RCCL) PyTorch has
already loaded. If the library is missing the import fails loudly: there is no fallback path.

`ddl_lib` (the reference's override, cpp_backend.py:34) selects another build: the tests, the
bench and smoke() load lib/libddl_amd_testing.so — the same engine objects plus the test /
measurement surface (include/ddl_amd_testing.h) — and the signatures of that surface are bound
only when the loaded library exports it.
"""
import ctypes
import os

import torch  # noqa: F401  (must precede the CDLL: one HIP runtime per process)

_PKG_ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
DEFAULT_LIB = os.path.join(_PKG_ROOT, 'lib', 'libddl_amd.so')
TESTING_LIB = os.path.join(_PKG_ROOT, 'lib', 'libddl_amd_testing.so')

# include/ddl_amd.h: what the deployment library exports (and nothing else)
DEPLOYMENT_API = (
    'ddl_version', 'ddl_build_info', 'ddl_last_error', 'ddl_dtype_name', 'ddl_dtype_size', 'ddl_get_unique_id',
    'ddl_init', 'ddl_init_single', 'ddl_control_listen', 'ddl_control_connect', 'ddl_control_stats', 'ddl_finalize',
    'ddl_is_initialized', 'ddl_set_config', 'ddl_get_config', 'ddl_comm_transport', 'communicator_rank',
    'communicator_size', 'world_communicator', 'split_communicator', 'detach_communicator', 'py_info', 'py_debug',
    'py_error', 'ddl_allreduce', 'ddl_allreduce_batch', 'ddl_broadcast', 'ddl_allgatherv', 'ddl_allgather',
    'ddl_allreduce_host', 'ddl_tune_result', 'ddl_allreduce_submit', 'ddl_broadcast_submit', 'ddl_allgather_submit',
    'ddl_allreduce_submit_batch', 'ddl_allreduce_submit_mem', 'ddl_allreduce_submit_batch_mem',
    'ddl_broadcast_submit_mem', 'ddl_allgather_submit_mem', 'ddl_wait_all', 'ddl_host_unregister',
    'ddl_kernel_timing', 'ddl_kernel_stats', 'ddl_completion_create', 'ddl_completion_slots', 'ddl_completion_done',
    'ddl_completion_wait', 'ddl_completion_poll', 'ddl_completion_destroy')

# enum ddl_dtype (tensorflow::DataType numbers, reference src/cpp/def.h:10-53)
DT_FLOAT, DT_DOUBLE, DT_INT32, DT_INT64, DT_BFLOAT16, DT_HALF, DT_UINT64 = 1, 2, 3, 9, 14, 19, 23
STATUS_OK = 0
STATUS_NAMES = {0: 'OK', 1: 'COMM_ERROR', 2: 'ERROR_UNKNOWN', 3: 'INVALID_ARGUMENT',
                4: 'UNSUPPORTED_DTYPE', 5: 'HIP_ERROR', 6: 'NOT_INITIALIZED', 7: 'DUPLICATE_KEY',
                8: 'CONFIG_MISMATCH'}
STATUS_CONFIG_MISMATCH = 8
OP_SUM = 0
MEMORY_DEVICE, MEMORY_HOST = 0, 1  # enum ddl_memory

DONE_FN = ctypes.CFUNCTYPE(None, ctypes.c_int, ctypes.c_void_p)
# ddl_alloc_fn: output allocation of a keyed allgather (first_dim, bytes, user) -> device pointer
ALLOC_FN = ctypes.CFUNCTYPE(ctypes.c_void_p, ctypes.c_size_t, ctypes.c_size_t, ctypes.c_void_p)


class DDLError(RuntimeError):
    """A non-OK status from the engine (StatusCode, reference src/cpp/def.h:70-74)."""

    def __init__(self, status: int, where: str, detail: str):
        self.status = status
        super().__init__(f'{where} failed: {STATUS_NAMES.get(status, status)}: {detail}')


class CPPBackend:
    """Manages the native engine (same role and names as the reference's CPPBackend)."""
    __path_to_lib = DEFAULT_LIB
    __initialized = False
    __c_api = None

    @classmethod
    def __initialize(cls, path_to_lib: str = None):
        if path_to_lib is None:
            path_to_lib = os.environ.get('ddl_lib')  # same override as the reference (:34)
        if path_to_lib is not None:
            cls.__path_to_lib = path_to_lib
        if not os.path.exists(cls.__path_to_lib):
            raise ImportError(
                f'ddl engine library not found at {cls.__path_to_lib}; build it with '
                f'`python -c "import __graft_entry__ as g; g.build()"` (no fallback exists)')
        lib = ctypes.CDLL(cls.__path_to_lib, mode=ctypes.RTLD_GLOBAL)
        missing = [n for n in DEPLOYMENT_API if not hasattr(lib, n)]
        if missing:
            raise ImportError(f'{cls.__path_to_lib} lacks the deployment C-ABI: {missing}')
        cid, sz, vp, ci = ctypes.c_longlong, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_int

        def sig(name, restype, *argtypes):
            f = getattr(lib, name, None)
            if f is None:  # a test / measurement entry point: not in the deployment library
                return
            f.restype = restype
            f.argtypes = list(argtypes)

        sig('ddl_version', ci)
        sig('ddl_last_error', ctypes.c_char_p)
        sig('ddl_dtype_size', sz, ci)
        sig('ddl_get_unique_id', ci, vp, sz)
        sig('ddl_init', ci, ci, ci, ci, vp, sz)
        sig('ddl_init_single', ci, ci)
        sig('ddl_control_listen', ci, ctypes.c_char_p, sz)
        sig('ddl_control_connect', ci, ctypes.c_char_p)
        sig('ddl_control_connect_ranked', ci, ci, ci, ctypes.c_char_p)
        sig('ddl_control_negotiate', ci, ctypes.c_char_p, ctypes.c_char_p, sz)
        sig('ddl_control_stats', ci, ctypes.POINTER(ctypes.c_longlong), ctypes.POINTER(ctypes.c_longlong))
        sig('ddl_allreduce_variant', ci, cid, vp, vp, sz, ci, ci, vp, ci)
        sig('ddl_comm_transport', ci, cid, ctypes.POINTER(ci), ctypes.POINTER(ci))
        sig('ddl_testing_round_log', ci, cid, ctypes.POINTER(ctypes.c_longlong), ctypes.POINTER(ctypes.c_longlong), ci,
            ctypes.POINTER(ci))
        sig('ddl_allreduce_host', ci, cid, vp, vp, sz, ci, ci)
        sig('ddl_ring_program', ci, ci, ci, sz, ci, ctypes.POINTER(ctypes.c_longlong), sz, ctypes.POINTER(sz))
        sig('ddl_finalize', ci)
        sig('ddl_is_initialized', ci)
        sig('ddl_set_config', ci, ctypes.c_char_p, ctypes.c_longlong)
        sig('ddl_get_config', ctypes.c_longlong, ctypes.c_char_p)
        # reference c_api.h:15-41 (ctypes signatures as cpp_backend.py:47-78)
        sig('communicator_rank', ci, cid)
        sig('communicator_size', ci, cid)
        sig('world_communicator', cid)
        sig('split_communicator', cid, cid, ci, ci)
        sig('detach_communicator', None, cid)
        sig('py_info', None, ctypes.c_char_p)
        sig('py_debug', None, ctypes.c_char_p)
        sig('py_error', None, ctypes.c_char_p)
        # data plane
        sig('ddl_allreduce', ci, cid, vp, vp, sz, ci, ci, vp)
        sig('ddl_allreduce_batch', ci, cid, ci, ctypes.POINTER(vp), ctypes.POINTER(vp), ctypes.POINTER(sz), ci, ci, vp)
        for name in ('ddl_local_allreduce_batch', 'ddl_testing_thread_allreduce_batch',
                     'ddl_rccl_loopback_allreduce_batch'):
            sig(name, ci, ci, ci, ctypes.POINTER(vp), ctypes.POINTER(vp), ctypes.POINTER(sz), ci, vp)
        sig('ddl_allreduce_submit', ci, cid, ctypes.c_char_p, vp, vp, sz, ci, ci, vp, DONE_FN, vp)
        sig('ddl_allreduce_submit_batch', ci, cid, ci, ctypes.POINTER(ctypes.c_char_p), ctypes.POINTER(vp),
            ctypes.POINTER(vp), ctypes.POINTER(sz), ctypes.POINTER(ci), ci, vp, DONE_FN, ctypes.POINTER(vp))
        sig('ddl_allreduce_submit_mem', ci, cid, ctypes.c_char_p, vp, vp, sz, ci, ci, ci, vp, DONE_FN, vp)
        sig('ddl_allreduce_submit_batch_mem', ci, cid, ci, ctypes.POINTER(ctypes.c_char_p), ctypes.POINTER(vp),
            ctypes.POINTER(vp), ctypes.POINTER(sz), ctypes.POINTER(ci), ci, ci, vp, DONE_FN, ctypes.POINTER(vp))
        sig('ddl_broadcast_submit_mem', ci, cid, ctypes.c_char_p, vp, vp, sz, ci, ci, ci, vp, DONE_FN, vp)
        sig('ddl_allgather_submit_mem', ci, cid, ctypes.c_char_p, vp, sz, sz, ci, ci, vp, ALLOC_FN, DONE_FN, vp)
        sig('ddl_control_channel_open', ctypes.c_longlong, ctypes.c_char_p, sz)
        sig('ddl_control_channel_connect', ci, ctypes.c_longlong, ci, ci, ctypes.c_char_p)
        sig('ddl_control_channel_negotiate', ci, ctypes.c_longlong, ctypes.c_char_p, ctypes.c_char_p, sz)
        sig('ddl_control_channel_close', ci, ctypes.c_longlong)
        sig('ddl_wait_all', ci, cid)
        sig('ddl_completion_create', vp, ci)
        sig('ddl_completion_slots', ci, vp, ci, ci, ctypes.POINTER(vp))
        sig('ddl_completion_done', None, ci, vp)
        sig('ddl_completion_wait', ci, vp, ci, ctypes.c_double, ctypes.POINTER(ci))
        sig('ddl_completion_poll', ci, vp, ctypes.POINTER(ci), ci)
        sig('ddl_completion_destroy', None, vp)
        sig('ddl_host_unregister', ci, ctypes.c_void_p, ctypes.c_size_t)
        sig('ddl_broadcast_submit', ci, cid, ctypes.c_char_p, vp, vp, sz, ci, ci, vp, DONE_FN, vp)
        sig('ddl_allgather_submit', ci, cid, ctypes.c_char_p, vp, sz, sz, ci, vp, ALLOC_FN, DONE_FN, vp)
        sig('ddl_broadcast', ci, cid, vp, sz, ci, ci, vp)
        sig('ddl_allgatherv', ci, cid, vp, sz, vp, ctypes.POINTER(sz), ctypes.POINTER(sz), ci, vp)
        sig('ddl_allgather', ci, cid, vp, sz, vp, sz, ci, vp)
        sig('ddl_local_broadcast', ci, ci, ci, ctypes.POINTER(vp), sz, ci, vp)
        sig('ddl_local_allgatherv', ci, ci, ctypes.POINTER(vp), ctypes.POINTER(vp), ctypes.POINTER(sz),
            ctypes.POINTER(sz), ci, vp)
        sig('ddl_broadcast_program', ci, ci, ci, ci, sz, ci, ctypes.POINTER(ctypes.c_longlong), sz,
            ctypes.POINTER(sz))
        sig('ddl_allgather_program', ci, ci, ci, ctypes.POINTER(sz), ctypes.POINTER(sz), ci,
            ctypes.POINTER(ctypes.c_longlong), sz, ctypes.POINTER(sz))
        sig('ddl_tune_result', ci, cid, sz, ctypes.POINTER(ci), ctypes.POINTER(ci),
            ctypes.POINTER(ctypes.c_longlong), ctypes.POINTER(ctypes.c_float), ci)
        sig('ddl_local_tune', ci, ci, sz, ci, vp, ctypes.POINTER(ci), ctypes.POINTER(ci),
            ctypes.POINTER(ctypes.c_longlong), ctypes.POINTER(ctypes.c_float), ci)
        sig('ddl_kernel_timing', ci, cid, ci)
        sig('ddl_kernel_stats', ci, cid, ctypes.POINTER(ctypes.c_longlong), ctypes.POINTER(ctypes.c_double),
            ctypes.POINTER(ctypes.c_double))
        sig('ddl_reduce_local', ci, vp, vp, sz, ci, vp)
        sig('ddl_reduce_sum2', ci, vp, vp, vp, sz, ci, vp)
        sig('ddl_reduce_sum2_variant', ci, ci, vp, vp, vp, sz, ci, vp)
        sig('ddl_reduce_fold', ci, vp, vp, ctypes.POINTER(vp), ci, sz, ci, vp)
        sig('ddl_reduce_fold_ordered', ci, vp, vp, ctypes.POINTER(vp), ci, sz, ci, ci, vp)
        sig('ddl_reduce_fold_batch', ci, ci, ctypes.POINTER(vp), ctypes.POINTER(vp), ctypes.POINTER(vp), ci,
            ctypes.POINTER(sz), ci, ci, vp)
        sig('ddl_pack', ci, vp, ctypes.POINTER(vp), ctypes.POINTER(sz), ci, vp)
        sig('ddl_unpack', ci, ctypes.POINTER(vp), vp, ctypes.POINTER(sz), ci, vp)
        sig('ddl_local_ring_allreduce', ci, ci, ctypes.POINTER(vp), ctypes.POINTER(vp), sz, ci, ci, vp)
        # RCCL loopback (test / diagnostic: the RCCL transport on one GPU)
        fp, lp = ctypes.POINTER(ctypes.c_float), ctypes.POINTER(ctypes.c_longlong)
        sig('ddl_testing_thread_allreduce', ci, ci, ctypes.POINTER(vp), ctypes.POINTER(vp), sz, ci, vp)
        sig('ddl_testing_thread_broadcast', ci, ci, ci, ctypes.POINTER(vp), sz, ci, vp)
        sig('ddl_testing_thread_allgatherv', ci, ci, ctypes.POINTER(vp), ctypes.POINTER(vp), ctypes.POINTER(sz),
            ctypes.POINTER(sz), ci, vp)
        sig('ddl_testing_drop_wait', ci, ci)
        sig('ddl_testing_control_fault', ci, ci)
        sig('ddl_testing_host_coll_fault', ci, ctypes.c_longlong)
        sig('ddl_testing_fold_variant', ci, ci)
        sig('ddl_testing_thread_transport', ci, ci, ctypes.POINTER(ctypes.c_longlong))
        sig('ddl_testing_dep_trace', ci, ci)
        sig('ddl_testing_thread_fused_allreduce', ci, ci, ci, ctypes.POINTER(vp), ctypes.POINTER(vp),
            ctypes.POINTER(sz), ci, vp, ctypes.POINTER(sz))
        sig('ddl_testing_dep_check', ci, lp, ctypes.c_char_p, sz)
        sig('ddl_rccl_loopback_init', ci, ci)
        sig('ddl_rccl_loopback_split', ci, ci, ci, ctypes.POINTER(ci), ctypes.POINTER(ci))
        sig('ddl_rccl_loopback_allreduce', ci, ci, ctypes.POINTER(vp), ctypes.POINTER(vp), sz, ci, vp)
        sig('ddl_rccl_loopback_broadcast', ci, ci, ci, ctypes.POINTER(vp), sz, ci, vp)
        sig('ddl_rccl_loopback_allgatherv', ci, ci, ctypes.POINTER(vp), ctypes.POINTER(vp), ctypes.POINTER(sz),
            ctypes.POINTER(sz), ci, vp)
        sig('ddl_rccl_loopback_allgather', ci, vp, vp, sz, vp)
        sig('ddl_rccl_loopback_max', ci, fp, ci, vp)
        sig('ddl_rccl_loopback_tune', ci, ci, sz, ci, vp, ctypes.POINTER(ci), ctypes.POINTER(ci), lp, fp, ci)
        sig('ddl_rccl_loopback_stats', ci, ci, lp)
        sig('ddl_rccl_loopback_finalize', ci)
        # schedule introspection
        sig('ddl_ring_count', ci, ci, ci)
        sig('ddl_ring_perm', ci, ci, ci, ci, ctypes.POINTER(ci))
        sig('ddl_chunk_range', ci, sz, ci, ci, ci, ci, ci, ctypes.POINTER(sz), ctypes.POINTER(sz))
        sig('ddl_ring_shape', ci, sz, ci, ci, ctypes.POINTER(ci), ctypes.POINTER(ci))
        sig('ddl_make_plans', ci, ctypes.POINTER(sz), ctypes.POINTER(sz), sz, sz, ctypes.POINTER(sz), sz,
            ctypes.POINTER(sz))
        cls.__c_api = lib
        cls.__initialized = True

    @classmethod
    def c_api(cls):
        if not cls.__initialized:
            cls.__initialize()
        return cls.__c_api

    @classmethod
    def has_testing_api(cls) -> bool:
        """Whether the loaded library is the testing build (include/ddl_amd_testing.h)."""
        return hasattr(cls.c_api(), 'ddl_init_test_transport')

    @classmethod
    def path(cls) -> str:
        cls.c_api()
        return cls.__path_to_lib


def check(status: int, where: str) -> None:
    """Raise DDLError for a non-OK status, with the engine's last error message."""
    if status != STATUS_OK:
        msg = CPPBackend.c_api().ddl_last_error()
        raise DDLError(status, where, msg.decode(errors='replace') if msg else '')
