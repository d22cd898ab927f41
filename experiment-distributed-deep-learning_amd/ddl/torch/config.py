"""Engine tunables from Python (ddl_set_config / ddl_get_config, include/ddl_amd.h).

The SHARED tunables (SHARED below) must be equal on every rank: the schedule, the fusion plans and
the summation order are collective decisions. The ranks agree on a hash of them at a
communicator's first collective and after any change (change them on every rank between the same
two collectives), and every keyed round carries it: a mismatch fails the collective or round on
every rank with CONFIG_MISMATCH instead of hanging. The other keys are per process. The reference has no tunables beyond its compiled
constants (MAX_MPI_BUFFER_SIZE, MPIBackend.h:12); the defaults reproduce its behaviour, with
`reference_order` = 1 making every sum bit-equal to its MPI_Allreduce.

    from ddl.torch import config
    config.set('fusion_threshold_bytes', 64 << 20)
    with config.override(tune=0, algo=1):
        ...
"""
import contextlib

from ddl.torch.cpp_backend import CPPBackend, check

KEYS = ('algo', 'slice_bytes', 'rings', 'max_slices', 'fusion_threshold_bytes', 'log_level', 'cycle_time_us',
        'host_chunk_bytes', 'host_copy_threads', 'host_zero_copy', 'tune', 'fusion_pipeline_bytes', 'one_rank_shortcut',
        'pipeline_rounds', 'reference_order', 'host_register_cache_bytes', 'capture_mode',
        'fold_form', 'compute_cu_mask', 'host_numa_bind', 'rccl_min_ctas', 'rccl_max_ctas', 'queue_isolation')
SHARED = ('algo', 'slice_bytes', 'rings', 'max_slices', 'fusion_threshold_bytes', 'tune', 'fusion_pipeline_bytes',
          'reference_order', 'host_chunk_bytes', 'rccl_min_ctas', 'rccl_max_ctas')


def set(key: str, value: int) -> None:  # noqa: A001 (mirrors ddl_set_config)
    """Set one tunable; raises DDLError for an unknown key or a rejected value."""
    check(CPPBackend.c_api().ddl_set_config(key.encode(), int(value)), f'ddl_set_config({key})')


def get(key: str) -> int:
    """Current value of one tunable (-1 for an unknown key, as ddl_get_config)."""
    return int(CPPBackend.c_api().ddl_get_config(key.encode()))


def snapshot() -> dict:
    return {k: get(k) for k in KEYS}


@contextlib.contextmanager
def override(**values):
    """Set tunables for a block and restore the previous values after it."""
    old = {k: get(k) for k in values}
    try:
        for k, v in values.items():
            set(k, v)
        yield
    finally:
        for k, v in old.items():
            set(k, v)
