"""The C-ABI library loads and exports every symbol include/ddl_amd.h declares; host-only
entry points behave (no GPU calls here)."""
import ctypes
import os
import re
import subprocess

import pytest

from conftest import PKG, ROOT

HEADER = os.path.join(ROOT, 'include', 'ddl_amd.h')
TESTING_HEADER = os.path.join(ROOT, 'include', 'ddl_amd_testing.h')
LIB = os.path.join(PKG, 'lib', 'libddl_amd.so')  # the deployment library
TESTING_LIB = os.path.join(PKG, 'lib', 'libddl_amd_testing.so')

# reference src/cpp/c_api.h:15-41 (the ctypes surface, cpp_backend.py:47-78)
REFERENCE_C_API = {'communicator_rank', 'communicator_size', 'world_communicator', 'split_communicator',
                   'detach_communicator', 'py_info', 'py_debug', 'py_error'}
# what a framework binding needs: lifecycle, tunables, the data plane, keyed requests, and the
# measurement hooks on a live communicator
DEPLOYMENT = {
    'ddl_version', 'ddl_build_info', 'ddl_last_error', 'ddl_dtype_name', 'ddl_dtype_size',
    'ddl_get_unique_id', 'ddl_init', 'ddl_init_single', 'ddl_control_listen', 'ddl_control_connect',
    'ddl_control_stats', 'ddl_finalize', 'ddl_is_initialized', 'ddl_set_config', 'ddl_get_config',
    'ddl_comm_transport', 'ddl_allreduce', 'ddl_allreduce_batch', 'ddl_broadcast', 'ddl_allgatherv', 'ddl_allgather',
    'ddl_allreduce_host', 'ddl_tune_result', 'ddl_allreduce_submit', 'ddl_broadcast_submit',
    'ddl_allgather_submit', 'ddl_allreduce_submit_batch', 'ddl_allreduce_submit_mem',
    'ddl_allreduce_submit_batch_mem', 'ddl_broadcast_submit_mem', 'ddl_allgather_submit_mem', 'ddl_wait_all', 'ddl_host_unregister',
    'ddl_kernel_timing', 'ddl_kernel_stats', 'ddl_completion_create', 'ddl_completion_slots', 'ddl_completion_done',
    'ddl_completion_wait', 'ddl_completion_poll', 'ddl_completion_destroy'}


def declared_functions(header=HEADER):
    text = open(header).read()
    text = re.sub(r'/\*.*?\*/', '', text, flags=re.S)
    text = '\n'.join(line for line in text.splitlines() if not line.lstrip().startswith('typedef'))
    names = re.findall(r'^[A-Za-z_][\w \*]*?\b([a-z_][a-z0-9_]*)\s*\(', text, flags=re.M)
    return sorted(set(names))


def test_header_declares_reference_c_api_names():
    names = declared_functions()
    assert REFERENCE_C_API <= set(names)
    assert 'ddl_allreduce' in names and 'ddl_allreduce_submit' in names


def test_deployment_header_is_only_the_deployment_surface():
    """include/ddl_amd.h declares the deployment surface plus the reference's
    c_api.h names and nothing else; the test transport, virtual-rank worlds, the RCCL loopback,
    raw kernels and introspection live in include/ddl_amd_testing.h."""
    names = set(declared_functions())
    assert names == DEPLOYMENT | REFERENCE_C_API, (sorted(names - DEPLOYMENT - REFERENCE_C_API),
                                                   sorted(DEPLOYMENT | REFERENCE_C_API - names))
    testing = set(declared_functions(TESTING_HEADER))
    assert not testing & names
    for n in ('ddl_init_test_transport', 'ddl_local_ring_allreduce', 'ddl_rccl_loopback_init', 'ddl_ring_program',
              'ddl_reduce_local', 'ddl_allreduce_variant', 'ddl_control_channel_open'):
        assert n in testing, n


def _exported(path):
    out = subprocess.run(['nm', '-D', '--defined-only', path], capture_output=True, text=True, check=True).stdout
    return set(line.split()[-1] for line in out.splitlines() if ' T ' in line)


def test_deployment_library_exports_exactly_the_header():
    """libddl_amd.so exports the functions include/ddl_amd.h declares and
    nothing else (version script ddl_amd.map): the reference's c_api.h names plus the deployment
    surface."""
    exported = _exported(LIB)
    declared = set(declared_functions())
    assert exported == declared, (sorted(exported - declared), sorted(declared - exported))
    dyn = subprocess.run(['nm', '-D', '--defined-only', LIB], capture_output=True, text=True, check=True).stdout
    assert all(line.split()[1] in 'T' for line in dyn.splitlines() if len(line.split()) == 3 and
               line.split()[1] not in 'Aw'), 'the deployment library exports data or weak symbols'


def test_torch_mirror_requires_exactly_the_deployment_surface():
    """The torch mirror refuses a library that lacks any deployment entry point, and its list is
    the header's (cpp_backend.DEPLOYMENT_API)."""
    from ddl.torch import cpp_backend
    assert set(cpp_backend.DEPLOYMENT_API) == set(declared_functions())


def test_testing_library_exports_both_headers():
    exported = _exported(TESTING_LIB)
    declared = declared_functions() + declared_functions(TESTING_HEADER)
    missing = [n for n in declared if n not in exported]
    assert not missing, f'declared but not exported: {missing}'


def test_deployment_library_links_no_test_harness():
    """The test worlds, the test transport, the RCCL loopback and the happens-before recorder are
    linked into the testing library only: not even a local symbol of theirs is in the deployment
    library (both are built from the same engine objects; the harness objects are extra)."""
    syms = subprocess.run(['nm', '-C', LIB], capture_output=True, text=True, check=True).stdout
    for name in ('ThreadFabric', 'ThreadWorld', 'LocalWorld', 'CallbackTransport', 'RcclLoopback',
                 'ddl_testing_', 'ddl_rccl_loopback', 'ddl_local_', 'dep::start', 'dep::check'):
        assert name not in syms, name
    tsyms = subprocess.run(['nm', '-C', TESTING_LIB], capture_output=True, text=True, check=True).stdout
    assert 'ThreadWorld' in tsyms and 'dep::check' in tsyms


def test_both_libraries_carry_identical_gpu_code():
    """The kernels the tests and the bench measure (testing library) are byte-for-byte the
    deployment library's: the same .hip_fatbin section (the gfx950 code objects)."""
    import tempfile
    blobs = []
    with tempfile.TemporaryDirectory() as d:
        for i, path in enumerate((LIB, TESTING_LIB)):
            out = os.path.join(d, f'{i}.bin')
            subprocess.run(['objcopy', '-O', 'binary', '--only-section=.hip_fatbin', path, out], check=True)
            blobs.append(open(out, 'rb').read())
    assert len(blobs[0]) > 100_000 and blobs[0] == blobs[1]


def test_same_build_id_in_both_libraries():
    from conftest import _library_build_id, source_hash
    assert _library_build_id(LIB) == _library_build_id(TESTING_LIB) == source_hash()


def test_test_transport_refused_without_opt_in(lib):
    """ddl_init_test_transport (host-synchronised groups, no RCCL) refuses unless the process
    opts in with DDL_ALLOW_TEST_TRANSPORT=1, so a binding cannot pick it up by mistake."""
    fn = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_longlong, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p)(
        lambda *a: 0)
    lib.ddl_init_test_transport.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, type(fn), ctypes.c_void_p,
                                            ctypes.c_void_p]
    old = os.environ.pop('DDL_ALLOW_TEST_TRANSPORT', None)
    try:
        assert lib.ddl_init_test_transport(0, 2, 0, fn, None, None) == 3
        assert b'DDL_ALLOW_TEST_TRANSPORT' in lib.ddl_last_error()
    finally:
        if old is not None:
            os.environ['DDL_ALLOW_TEST_TRANSPORT'] = old


def test_library_loads_via_ctypes_and_reports(lib):
    assert lib.ddl_version() >= 1
    assert lib.ddl_dtype_size(1) == 4 and lib.ddl_dtype_size(19) == 2 and lib.ddl_dtype_size(23) == 8
    assert lib.ddl_dtype_size(7) == 0  # DT_STRING unsupported


def test_uninitialized_world_is_an_error_not_a_crash(lib):
    if lib.ddl_is_initialized():
        pytest.skip('world already initialized in this process')
    assert lib.world_communicator() == 0
    assert b'ddl_init' in lib.ddl_last_error()
    assert lib.communicator_rank(12345) == -1


def test_config_roundtrip(lib):
    old = lib.ddl_get_config(b'slice_bytes')
    assert lib.ddl_set_config(b'slice_bytes', 1 << 20) == 0
    assert lib.ddl_get_config(b'slice_bytes') == 1 << 20
    assert lib.ddl_set_config(b'slice_bytes', old) == 0
    assert lib.ddl_set_config(b'no_such_key', 1) == 3
    assert lib.ddl_set_config(b'fusion_threshold_bytes', 0) == 3
    # the product default: sums bit-equal to the reference's MPI_Allreduce
    assert lib.ddl_get_config(b'reference_order') == 1
    # keyed rounds pipelined by default (done() fired by the completion thread)
    assert lib.ddl_get_config(b'pipeline_rounds') == 1
    # captures post serially by default (2: single-stream DAG); r03's forked mode 1 and its
    # capture_forked key are refused since r04 (the HIP runtime crashed on them)
    assert lib.ddl_get_config(b'capture_mode') == 0
    assert lib.ddl_set_config(b'capture_mode', 3) == 3
    assert lib.ddl_set_config(b'capture_mode', 1) == 3 and b'removed' in lib.ddl_last_error()
    assert lib.ddl_set_config(b'capture_forked', 1) == 3
    assert lib.ddl_get_config(b'capture_forked') == -1
    assert lib.ddl_set_config(b'capture_mode', 2) == 0 and lib.ddl_get_config(b'capture_mode') == 2
    assert lib.ddl_set_config(b'capture_mode', 0) == 0
    # multi-rank compute streams on every CU by default (8 / 4 / 2: leave every n-th to RCCL)
    assert lib.ddl_get_config(b'compute_cu_mask') == 0
    assert lib.ddl_set_config(b'compute_cu_mask', 3) == 3
    for v in (2, 4, 8, 0):
        assert lib.ddl_set_config(b'compute_cu_mask', v) == 0 and lib.ddl_get_config(b'compute_cu_mask') == v
    # RCCL communicator CTA bounds (ncclConfig_t.minCTAs / maxCTAs): 0 = RCCL's default
    for key in (b'rccl_min_ctas', b'rccl_max_ctas'):
        assert lib.ddl_get_config(key) == 0
        assert lib.ddl_set_config(key, -1) == 3 and lib.ddl_set_config(key, 257) == 3
        for v in (1, 32, 256, 0):
            assert lib.ddl_set_config(key, v) == 0 and lib.ddl_get_config(key) == v
    # hardware-queue classes of multi-rank communicators' streams: off by default, local, 0 / 1
    assert lib.ddl_get_config(b'queue_isolation') == 0
    for v in (1, 0):
        assert lib.ddl_set_config(b'queue_isolation', v) == 0 and lib.ddl_get_config(b'queue_isolation') == v
    # the fold's form: 0 auto (default), 1 tile, 2 run
    assert lib.ddl_get_config(b'fold_form') == 0
    assert lib.ddl_set_config(b'fold_form', 3) == 3
    # the measured losers of r03 are gone: quarter-chunk tapers, direct DMA
    for gone in (b'host_taper', b'host_direct_dma'):
        assert lib.ddl_set_config(gone, 0) == 3 and lib.ddl_get_config(gone) == -1


def test_product_does_not_reference_oracle():
    """The product path never loads or names the oracle (it is test infrastructure)."""
    for d, _, files in os.walk(PKG):
        for f in files:
            if f.endswith(('.cpp', '.h', '.hip', '.py')):
                text = open(os.path.join(d, f), errors='replace').read()
                assert 'ddl_oracle' not in text and 'ddlo_' not in text, f
    for path in (LIB, TESTING_LIB):
        out = subprocess.run(['readelf', '-d', path], capture_output=True, text=True, check=True).stdout
        assert 'oracle' not in out


def test_rccl_channel_bounds_from_the_environment():
    """DDL_RCCL_MIN_CTAS / DDL_RCCL_MAX_CTAS seed rccl_min_ctas / rccl_max_ctas (clamped to 0..256),
    DDL_QUEUE_ISOLATION queue_isolation, for a deployment that sets them per job; read in a fresh process (the config is built once)."""
    import sys
    code = ('import ctypes; l = ctypes.CDLL(%r); l.ddl_get_config.restype = ctypes.c_longlong; '
            'print(l.ddl_get_config(b"rccl_min_ctas"), l.ddl_get_config(b"rccl_max_ctas"), '
            'l.ddl_get_config(b"queue_isolation"))' % LIB)
    env = dict(os.environ, DDL_RCCL_MIN_CTAS='12', DDL_RCCL_MAX_CTAS='999', DDL_QUEUE_ISOLATION='1')
    out = subprocess.run([sys.executable, '-c', code], env=env, capture_output=True, text=True, check=True).stdout
    assert out.split() == ['12', '256', '1'], out


def test_python_config_module(lib):
    """ddl.torch.config: every documented key reads back, override() restores, bad keys raise."""
    from ddl.torch import config
    from ddl.torch.cpp_backend import DDLError
    snap = config.snapshot()
    assert all(v >= 0 for v in snap.values()), snap
    assert snap['reference_order'] == 1
    with config.override(reference_order=0, slice_bytes=1 << 20):
        assert config.get('reference_order') == 0 and config.get('slice_bytes') == 1 << 20
    assert config.snapshot() == snap
    with pytest.raises(DDLError):
        config.set('no_such_key', 1)


def test_library_is_built_from_these_sources(lib):
    """ddl_build_info() carries the sha1 of the engine sources the library was compiled from;
    it must be this tree's (conftest rebuilds a stale library before any test runs)."""
    import conftest
    lib.ddl_build_info.restype = ctypes.c_char_p
    info = lib.ddl_build_info().decode()
    assert info == f'src={conftest.source_hash()} arch=gfx950', info


def _host_cuts(lib, total, chunk):
    n = ctypes.c_size_t(0)
    assert lib.ddl_testing_host_chunk_cuts(ctypes.c_size_t(total), ctypes.c_size_t(chunk), None,
                                           ctypes.c_size_t(0), ctypes.byref(n)) == 0, lib.ddl_last_error()
    buf = (ctypes.c_size_t * n.value)()
    assert lib.ddl_testing_host_chunk_cuts(ctypes.c_size_t(total), ctypes.c_size_t(chunk), buf, ctypes.c_size_t(n.value),
                                           ctypes.byref(n)) == 0, lib.ddl_last_error()
    return list(buf)


@pytest.mark.parametrize('chunk', [4096, 1 << 20, 32 << 20, 768])
def test_host_chunk_cuts(lib, chunk):
    """Host-staged transfers (ddl_allreduce_host, keyed host plans) cut whole chunks, the last one
    short. Every boundary but the end is a multiple of 256 (the dtype size divides 256), so every
    element lies in one chunk and ranks cut alike."""
    lib.ddl_testing_host_chunk_cuts.argtypes = [ctypes.c_size_t, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_size_t,
                                                ctypes.c_void_p]
    for total in [1, 256, chunk - 8, chunk, chunk + 256, 2 * chunk, 2 * chunk + 256, 3 * chunk, 3 * chunk + 1024,
                  8 * chunk, 8 * chunk + 4, 73 * chunk + 12345]:
        cuts = _host_cuts(lib, total, chunk)
        assert cuts[0] == 0 and cuts[-1] == total
        sizes = [b - a for a, b in zip(cuts, cuts[1:])]
        assert all(s > 0 for s in sizes)
        assert all(c % 256 == 0 for c in cuts[:-1])
        for a, s in zip(cuts, sizes):
            assert s == min(chunk, total - a), (total, a, s)
    assert _host_cuts(lib, 256 << 20, 32 << 20) == [k * (32 << 20) for k in range(9)]
    assert lib.ddl_testing_host_chunk_cuts(ctypes.c_size_t(1024), ctypes.c_size_t(100), None, ctypes.c_size_t(0),
                                           ctypes.byref(ctypes.c_size_t())) != 0


def test_host_tensor_finalizer_unregisters_its_range(lib, monkeypatch):
    """The torch mirror's side of the registration cache contract (ddl_host_unregister):
    with host_register_cache_bytes > 0 every host tensor a keyed request uses gets a finalizer on
    its STORAGE that hands the storage's range to ddl_host_unregister when the storage dies (after
    its last view, not before); a storage resized in place (its memory moved) has its old range
    released at its next submission, and so has a recorded range that a new storage now overlaps.
    With the cache off nothing is watched. CPU only: the calls are recorded through a wrapper of
    the library (no communicator is needed for a no-op)."""
    import gc

    import torch

    from ddl.torch import tensor_communicate as tc
    from ddl.torch.cpp_backend import CPPBackend
    assert lib.ddl_host_unregister(None, 0) == 0  # no handler, nothing cached: a no-op
    calls = []

    class Recording:
        def __getattr__(self, name):
            return getattr(lib, name)

        def ddl_host_unregister(self, ptr, nbytes):
            calls.append((ptr, nbytes))
            return lib.ddl_host_unregister(ptr, nbytes)
    monkeypatch.setattr(CPPBackend, 'c_api', staticmethod(lambda: Recording()))
    old = lib.ddl_get_config(b'host_register_cache_bytes')

    def rng(t):
        st = t.untyped_storage()
        return st.data_ptr(), st.nbytes()
    try:
        assert lib.ddl_set_config(b'host_register_cache_bytes', 0) == 0
        t = torch.zeros(1 << 16)
        tc._watch_host([t])
        assert not tc._watched  # cache off: not watched
        assert lib.ddl_set_config(b'host_register_cache_bytes', 1 << 30) == 0
        a, b = torch.zeros(1 << 16), torch.ones(3, 5)
        ra, rb = rng(a), rng(b)
        view = b[1:]  # a view: its storage is b's
        tc._watch_host([a, view, a])  # the same storage twice: one entry
        assert set(tc._watched) == {ra[0], rb[0]}
        del a, view
        gc.collect()
        assert calls == [ra], calls  # a's storage died; b's lives on
        del b
        gc.collect()
        assert calls == [ra, rb], calls
        assert not tc._watched
        # a storage resized in place: its old memory is released at its next submission
        c = torch.zeros(1 << 10)
        tc._watch_host([c])
        rc_old = rng(c)
        c.resize_(1 << 20)
        assert rng(c)[0] != rc_old[0]
        calls.clear()
        tc._watch_host([c])
        assert calls == [rc_old], calls
        assert set(tc._watched) == {rng(c)[0]}
        del c
        gc.collect()
        assert not tc._watched
    finally:
        lib.ddl_set_config(b'host_register_cache_bytes', old)
