#!/usr/bin/env python3
"""Benchmark of the gradient-bucket allreduce engine (BASELINE.json metric:
"device-resident allreduce GiB/s vs bucket size at 1/2/4/8 MI355X").

    python bench.py --gpus N --steps K --warmup W
    (N > 1: python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N ...)

A step is one pass of the hot path over one bucket resident in HBM:
  * N = 1 (BASELINE configs[1], "1xMI355X: local reduce kernel only, fp32 bucket sweep"): the
    per-hop reduce kernel acc += in over a 256 MiB fp32 bucket; value = bucket GiB/s. A sweep
    4 KiB..1 GiB of the same kernel is reported beside it.
  * N > 1 (configs[2], 8xMI355X fp32 256 MiB bucket): one ddl_allreduce of every rank's bucket
    (autotuned reduce-scatter / allgather over RCCL send/recv, HIP fold kernel, sums in MPICH's
    order); value = allreduce algbw = bucket GiB / max-over-ranks step time (nccl-tests
    convention), with busbw = 2(P-1)/P x algbw and its fraction of the link ceiling beside it.
    RCCL's own ncclAllReduce is timed on the same buffers as a comparator.
rank 0 prints ONE JSON line.
"""
import argparse
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(ROOT, 'experiment-distributed-deep-learning_amd')
sys.path.insert(0, PKG)
# the testing build of the engine (lib/libddl_amd_testing.so: the deployment library's engine
# objects and GPU code, byte for byte, plus the raw-kernel / comparator / test-transport entry
# points the measurement legs call), through the reference's `ddl_lib` override
os.environ.setdefault('ddl_lib', os.path.join(PKG, 'lib', 'libddl_amd_testing.so'))

GiB = float(1 << 30)
HBM_PEAK_GBS = 8000.0         # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
HBM_MEASURED_GBS = 6290.0     # same doc: 6.29 TB/s measured float4 copy
XGMI_LINK_GBS = 153.0         # task brief: per-link xGMI, 7 links per GPU
DT_FLOAT = 1


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--steps', type=int, default=50)
    ap.add_argument('--warmup', type=int, default=10)
    ap.add_argument('--bucket-mib', type=int, default=256)
    ap.add_argument('--no-cta-sweep', action='store_true', help='N>1: skip the RCCL channel-bound sweep')
    ap.add_argument('--no-sweep', action='store_true')
    ap.add_argument('--no-variants', action='store_true')
    ap.add_argument('--no-cpu-baseline', action='store_true')
    ap.add_argument('--no-host', action='store_true', help='skip the host-resident (PCIe) measurement')
    ap.add_argument('--no-fusion', action='store_true', help='skip the C5 many-bucket fusion measurement')
    ap.add_argument('--no-forced-data-plane', action='store_true',
                    help='N=1: skip the C5 legs that force the keyed data plane (profiling: keeps one pack '
                         'shape per kernel)')
    ap.add_argument('--no-host-steady', action='store_true',
                    help='N=1: skip the pageable host C5 leg over consecutive fresh / reused tensor sets')
    ap.add_argument('--no-c4', action='store_true', help='N>1: skip the C4 fp16 64 x 16 MiB measurement')
    ap.add_argument('--no-collectives', action='store_true', help='N>1: skip broadcast/allgather timing')
    ap.add_argument('--no-config-sweep', action='store_true', help='N>1: skip the ring config sweep')
    ap.add_argument('--no-size-sweep', action='store_true', help='N>1: skip the bucket-size sweep (ours vs RCCL)')
    ap.add_argument('--size-sweep-max-mib', type=int, default=1024, help='N>1: largest bucket of the size sweep')
    ap.add_argument('--rehearse', action='store_true',
                    help='N>1 on ONE GPU: run every leg with the point-to-point groups over gloo host copies '
                         '(test-harness transport, tools/gloo_transport.py) instead of RCCL; exercises the '
                         'bench code, its numbers are not measurements')
    ap.add_argument('--rehearse-rccl', action='store_true',
                    help='N>1 on ONE GPU over REAL multi-rank RCCL communicators: every rank gets its own '
                         'NCCL_HOSTID, so RCCL accepts N ranks on one device and connects them with its socket '
                         'transport over loopback; the node\'s code path end to end, its numbers are a socket\'s')
    ap.add_argument('--watchdog-s', type=float, default=420.0, help='N>1: abort a hung run after this')
    ap.add_argument('--force-multi', action='store_true', help='run the N>1 code path even at world size 1')
    ap.add_argument('--cpu-seconds', type=float, default=6.0)
    ap.add_argument('--variant', type=int, default=-1,
                    help='reduce kernel variant bits (-1 default; 1 nt-load a, 2 nt-load b, 4 nt-store, 8 lds b, '
                         '16 write-through store)')
    return ap.parse_args()


def dispatch_us(workload_key):
    """rocprofv3's average dispatch duration (us) of a bench leg's kernel, from the committed
    kernel trace of the same bench command (profiles/kernel_dispatch_us.json), with its source."""
    path = os.path.join(ROOT, 'profiles', 'kernel_dispatch_us.json')
    try:
        with open(path) as f:
            d = json.load(f)
    except (OSError, ValueError):
        return None
    e = d.get(workload_key)
    return None if e is None else dict(e, source=d.get('_source'))


def pmc_traffic(workload_key):
    """HBM bytes per launch from the committed rocprofv3 PMC summary (profiles/), if any."""
    path = os.path.join(ROOT, 'profiles', 'pmc_traffic.json')
    try:
        with open(path) as f:
            return json.load(f).get(workload_key)
    except (OSError, ValueError):
        return None


def cpu_reduce_port(n_bytes_sample, seconds):
    """The oracle's MPI_SUM restatement (oracle/ddl_oracle.c, 1 thread) on a bounded sample of
    the N=1 kernel workload: acc += in over a fp32 bucket of n_bytes_sample, repeated ~`seconds`
    (what MPICH's reduction op does per hop on the CPU; not the reference's whole path)."""
    import numpy as np
    lib = ctypes.CDLL(os.path.join(ROOT, 'oracle', 'build', 'libddl_oracle.so'))
    lib.ddlo_reduce_reps.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
    n = n_bytes_sample // 4
    rng = np.random.default_rng(1234)
    acc = rng.uniform(-1, 1, n).astype(np.float32)
    inp = rng.uniform(-1, 1, n).astype(np.float32)
    lib.ddlo_reduce_reps(DT_FLOAT, acc.ctypes.data, inp.ctypes.data, n, 1)  # first touch
    t0 = time.perf_counter()
    lib.ddlo_reduce_reps(DT_FLOAT, acc.ctypes.data, inp.ctypes.data, n, 1)
    one = max(time.perf_counter() - t0, 1e-6)
    reps = max(1, int(seconds / one))
    t0 = time.perf_counter()
    lib.ddlo_reduce_reps(DT_FLOAT, acc.ctypes.data, inp.ctypes.data, n, reps)
    dt = time.perf_counter() - t0
    return {'value': round(n_bytes_sample * reps / dt / GiB, 3), 'unit': 'GiB/s', 'cores': 1, 'kind': 'port',
            'sample': f'oracle ddlo_sum2 acc+=in, fp32 {n_bytes_sample >> 20} MiB x {reps} reps '
                      f'({dt:.1f} s, 1 thread) — restatement of MPICH MPI_SUM, the per-element op only'}


def _ref_path_leg(P, n, ntens, reps, timeout=180):
    """One run of oracle/ref_path_port.c (the reference's CPU path: handler send/recv threads,
    3-lap token, fusion memcpy, MPI_Allreduce) under MPICH with P ranks on the host cores."""
    import shutil
    import subprocess
    exe = os.path.join(ROOT, 'oracle', 'build', 'ref_path_port')
    mpiexec = '/opt/conda/bin/mpiexec'
    if not (os.path.exists(exe) and shutil.which(mpiexec)):
        return {'error': 'MPICH or oracle/build/ref_path_port missing on this host'}
    env = dict(os.environ)
    env['LD_LIBRARY_PATH'] = '/opt/conda/lib:' + env.get('LD_LIBRARY_PATH', '')
    env.setdefault('TMPDIR', '/tmp')
    try:
        p = subprocess.run([mpiexec, '-n', str(P), exe, str(n), str(ntens), str(reps)], capture_output=True,
                           text=True, timeout=timeout, env=env)
        r = json.loads(p.stdout.strip().splitlines()[-1]) if p.returncode == 0 else {'error': p.stderr[-300:]}
    except Exception as e:  # never let the baseline leg break the bench line
        r = {'error': repr(e)}
    r['cores'] = P * 3  # threads: main + handler send + handler recv per rank
    return r


def host_info():
    """What BASELINE.md asks a CPU baseline to state: the host's CPU model, its logical CPUs, the
    share this job may use (cgroup quota) and the MPI implementation the restated path runs on."""
    import subprocess
    model = None
    try:
        with open('/proc/cpuinfo') as f:
            for line in f:
                if line.startswith('model name'):
                    model = line.split(':', 1)[1].strip()
                    break
    except OSError:
        pass
    mpi = None
    try:
        p = subprocess.run(['/opt/conda/bin/mpichversion'], capture_output=True, text=True, timeout=20)
        for line in p.stdout.splitlines():
            if line.startswith('MPICH Version'):
                mpi = 'MPICH ' + line.split(':', 1)[1].strip()
            elif line.startswith('MPICH Device') and mpi:
                mpi += ' (' + line.split(':', 1)[1].strip() + ')'
    except (OSError, subprocess.SubprocessError):
        pass
    cg = cgroup_cpu()
    return {'cpu_model': model, 'nproc': os.cpu_count(), 'quota_cores': cg['quota_cores'] if cg else None,
            'mpi': mpi}


def cpu_baseline(P=2, reps=8):
    """cpu_baseline (the reference's own CPU+MPI loopback path on this box's host cores): the C3
    bucket shape (256 MiB fp32) through oracle/ref_path_port.c at P MPI ranks — the reference's
    handler threads, 3-lap token, fusion memcpy and MPI_Allreduce — best of `reps` after a
    warm-up (~10 s of CPU work at P = 2). The N = 1 line uses P = 2 (the smallest exchange), an
    N > 1 line P = N: the same ranks as its device run."""
    r = _ref_path_leg(P, 64 << 20, 1, reps)
    info = host_info()
    if 'GiBs' not in r:
        return {'value': None, 'unit': 'GiB/s', 'cores': r.get('cores'), 'kind': 'port', 'error': r.get('error'),
                **info}
    return {'value': r['GiBs'], 'unit': 'GiB/s', 'cores': r['cores'], 'kind': 'port', 'P': P,
            'sample': f'reference CPU path restated (oracle/ref_path_port.c): one 256 MiB fp32 bucket, {P} MPICH '
                      f'ranks x 3 threads, best {r["best_ms"]} ms of {reps} (mean {r["mean_ms"]} ms)',
            **info}


def cpu_reference_path():
    """The reference's whole CPU+MPI loopback path (oracle/ref_path_port.c: per-communicator
    send / recv handler threads with the cond-var token queue, 3-lap ring token over MPI p2p,
    fusion memcpy, MPI_Allreduce, per-round log lines) under MPICH with P ranks on the host
    cores: C1 (fp32[1024]) at P = 2 and 8, the C3 bucket shape (256 MiB fp32) at
    P = 8, and a bounded C5-like many-tensor sample (fp32 only: the reference rejects fp16) at
    P = 8. About 10-20 s."""
    res = {'kind': 'port', **host_info(),
           'what':'oracle/ref_path_port.c: reference handler threads + token ring + fusion + MPI_Allreduce '
                   '(MPICH 3.3.2 loopback), 3 threads per rank'}
    legs = (('C1_fp32_1024_P2', 2, 1024, 1, 200), ('C1_fp32_1024_P8', 8, 1024, 1, 100),
            ('C3shape_fp32_256MiB_P8', 8, 64 << 20, 1, 2), ('C5like_fp32_512x256KiB_P8', 8, 64 << 10, 512, 2))
    for tag, P, n, ntens, reps in legs:
        res[tag] = _ref_path_leg(P, n, ntens, reps)
    return res


NSETS = 3  # rotating buffer sets: >= 2 x 768 MiB of traffic between reuses of one set, so the
           # 256 MiB Infinity Cache cannot serve a re-read (MI355X_MICROARCH.md §Infinity Cache)
VARIANTS = {'default': -1, 'plain': 0, 'nt_load_a': 1, 'nt_load_ab': 3, 'nt_all': 7, 'lds_stage_b': 8,
            'lds_stage_b_nt_a': 9, 'wt_store': 16, 'nt_load_ab_wt_store': 19,
            # run form (bit 32: 8-tile runs per workgroup, a then b; bit 64: 4-tile runs), r05 A/B
            'run8_nt_all': 32 | 7, 'run8_nt_load_ab_wt_store': 32 | 19, 'run4_nt_all': 96 | 7,
            'run4_nt_load_ab_wt_store': 96 | 19}


GRAPH_SWEEP_MAX = 8 << 20  # sweep points also timed as hipGraph replays (launch-bound sizes)


def graph_reduce_us(lib, bufs, m, variant, per_graph=64, replays=20):
    """Per-bucket time of `per_graph` reduce launches captured into one hipGraph (torch.cuda.graph
    on a side stream: hipStreamBeginCapture) and replayed: the kernels back to back with no host
    launch in between — what a captured training step gets for its small buckets."""
    import torch
    from ddl.torch.cpp_backend import check
    gs = torch.cuda.Stream()
    graph = torch.cuda.CUDAGraph()
    torch.cuda.synchronize()
    with torch.cuda.graph(graph, stream=gs):
        for i in range(per_graph):
            acc, inp = bufs[i % len(bufs)]
            check(lib.ddl_reduce_sum2_variant(variant, acc.data_ptr(), acc.data_ptr(), inp.data_ptr(), m, DT_FLOAT,
                                              gs.cuda_stream), 'ddl_reduce_sum2_variant (captured)')
    best = float('inf')
    for _ in range(3):
        with torch.cuda.stream(gs):
            graph.replay()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(gs)
            for _ in range(replays):
                graph.replay()
            e1.record(gs)
        torch.cuda.synchronize()
        best = min(best, e0.elapsed_time(e1) * 1e3 / (replays * per_graph))
    del graph
    return best


def single_gpu(args):
    import torch
    from ddl.torch.cpp_backend import CPPBackend, check
    lib = CPPBackend.c_api()
    dev = torch.device('cuda', 0)
    torch.cuda.set_device(dev)
    S = args.bucket_mib << 20
    n = S // 4
    g = torch.Generator(device=dev).manual_seed(1234)
    sets = [((torch.rand(n, device=dev, generator=g) * 2 - 1), (torch.rand(n, device=dev, generator=g) * 2 - 1))
            for _ in range(NSETS)]
    stream = torch.cuda.current_stream(dev)
    sh = stream.cuda_stream
    counter = [0]

    def step(m=n, variant=args.variant, bufs=sets):
        acc, inp = bufs[counter[0] % len(bufs)]
        counter[0] += 1
        check(lib.ddl_reduce_sum2_variant(variant, acc.data_ptr(), acc.data_ptr(), inp.data_ptr(), m, DT_FLOAT, sh),
              'ddl_reduce_sum2_variant')

    def timed_kernel_ms(reps, **kw):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(reps):
            step(**kw)
        e1.record(stream)
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / reps

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record(stream)
    for _ in range(args.steps):
        step()
    ev1.record(stream)
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    kernel_ms = ev0.elapsed_time(ev1) / args.steps  # HIP events on the launch stream
    ms_per_step = wall * 1e3 / args.steps
    value = S / GiB / (ms_per_step / 1e3)
    achieved = 3.0 * S / (kernel_ms / 1e3) / 1e9

    extra = {}
    if not args.no_variants:  # interleaved rounds in one process (guide §5.4 rule 24)
        best = {k: float('inf') for k in VARIANTS}
        for _ in range(3):
            for k, v in VARIANTS.items():
                best[k] = min(best[k], timed_kernel_ms(12, variant=v))
        extra['variants_achieved_GBs'] = {k: round(3.0 * S / (t / 1e3) / 1e9, 1) for k, t in best.items()}

    if not args.no_sweep:
        sweep = []
        size = 4 << 10
        while size <= (1 << 30):
            m = size // 4
            bufs = [(torch.zeros(m, device=dev), torch.ones(m, device=dev)) for _ in range(NSETS)]
            reps = int(min(3000, max(6, (256 << 20) // size)))
            for _ in range(3):
                step(m=m, bufs=bufs)
            t = min(timed_kernel_ms(reps, m=m, bufs=bufs) for _ in range(3)) / 1e3  # best of 3 rounds
            point = {'bytes': size, 'us': round(t * 1e6, 2), 'bucket_GiBs': round(size / t / GiB, 2),
                     'hbm_GBs': round(3 * size / t / 1e9, 1)}
            if size <= GRAPH_SWEEP_MAX:  # launch-bound sizes: the same launches replayed from a hipGraph
                tg = graph_reduce_us(lib, bufs, m, args.variant) / 1e6
                point.update(graph_us=round(tg * 1e6, 2), graph_bucket_GiBs=round(size / tg / GiB, 2))
            sweep.append(point)
            del bufs
            size *= 2  # 4 KiB * 2^k up to 1 GiB, 19 points
        extra['sweep_fp32'] = sweep

    # the direct schedule's fold at P = 8 (chunk = S/8, 7 received inputs) and the per-hop
    # reduce in the C4 dtypes, on the same rotating-buffer discipline
    if not args.no_variants:
        extra['fold_kernel'] = fold_roofline(lib, dev, sh, S)
        # the fold the reference-order direct schedule runs at P = 8 (MPICH's pre-fold + tree)
        extra['fold_kernel_reference_order'] = fold_roofline(lib, dev, sh, S, order=1)
        # A/B: the same chunk in the tile form (every workgroup reads one tile of all 8 inputs at
        # once) instead of the run form (one input at a time over 16 KiB runs)
        extra['fold_kernel_tile_form'] = fold_roofline(lib, dev, sh, S, form=1)
        # C4's fold: one 16 MiB fp16 bucket at P = 8 is a 2 MiB chunk with 7 received inputs (fp16
        # widened to fp32, one rounding), measured two ways:
        #  * cache-resident: 2 operand sets = 36 MiB, inside the 256 MiB Infinity Cache — the
        #    direct schedule's situation (RCCL has just written the received slices). Not an HBM
        #    measurement: no fraction of HBM peak. Twice on fresh buffers; `us` is the mean of
        #    every replay round (the process's first fp16 graph reads slower on some boxes);
        #  * HBM-resident: 24 operand sets = 432 MiB rotating launch by launch, beyond the Infinity
        #    Cache. The chunk is 2 MiB - 4 KiB (1023 workgroups instead of 1025) so rocprofv3's
        #    per-(kernel, grid) split tells the two legs apart; the fraction of HBM peak is quoted
        #    on this one.
        # Beside each replay time: rocprofv3's per-dispatch average for the same (kernel, grid) from
        # the committed profile of this bench command (profiles/kernel_dispatch_us.json); the two
        # clocks differ for a 3-5 us kernel (DESIGN §5.2 reconciles them)
        c4a = fold_roofline(lib, dev, sh, 16 << 20, half=True)
        c4b = fold_roofline(lib, dev, sh, 16 << 20, half=True)
        rounds = c4a['rounds_us'] + c4b['rounds_us']
        mean_us = sum(rounds) / len(rounds)
        extra['fold_kernel_fp16_c4_cache_resident'] = dict(
            c4a, us=round(mean_us, 2), rounds_us=rounds,
            achieved_GBs=round(c4a['algorithmic_bytes_per_launch'] / mean_us / 1e3, 1), frac_of_peak=None,
            residency='Infinity Cache (36 MiB working set): not an HBM measurement',
            rocprof_dispatch_us=dispatch_us('fold_fp16_P8_C4_chunk_cache'),
            timing='mean of 2 x 3 replay rounds, 20 launches each, captured into a hipGraph, HIP events on the '
                   'replay stream')
        c4h = fold_roofline(lib, dev, sh, 16 << 20, half=True, nsets=24, chunk_bytes=(2 << 20) - 4096)
        c4h.update(residency='HBM (24 rotating operand sets, 432 MiB working set)',
                   rocprof_dispatch_us=dispatch_us('fold_fp16_P8_C4_chunk_hbm'))
        extra['fold_kernel_fp16_c4'] = c4h
        # ... and C4's 64 buckets folded the way the grouped allreduce folds them (ddl_allreduce_batch):
        # 8 buckets' chunks per launch (FoldBatch), 8 launches over the 64 buckets (1.2 GB of
        # operands: HBM, not the Infinity Cache)
        extra['fold_kernel_fp16_c4_batch'] = fold_batch_roofline(lib, dev, sh)
        extra['reduce_half_dtypes_achieved_GBs'] = half_dtypes(lib, dev, sh, S)

    traffic = pmc_traffic(f'reduce_fp32_{args.bucket_mib}MiB')
    out = {
        'metric': 'device-resident allreduce GiB/s vs bucket size at 1/2/4/8 MI355X',
        'value': round(value, 2),
        'unit': 'GiB/s',
        'n_gpus': 1,
        'steps': args.steps,
        'warmup': args.warmup,
        'ms_per_step': round(ms_per_step, 4),
        'higher_is_better': True,
        'scaling': 'weak',
        'vs_baseline': None,
        'dtype': 'f32',
        'data': f'synthetic U(-1,1) fp32 buckets resident in HBM, {NSETS} rotating buffer sets',
        'config': {'workload': 'C2: local reduce kernel acc += in (per-hop ring reduce), fp32, '
                               f'{args.bucket_mib} MiB bucket, 1xMI355X',
                   'bucket_bytes': S, 'parallelism': 'none (1 GPU)'},
        'roofline': {'bound': 'hbm', 'achieved': round(achieved, 1), 'peak': HBM_PEAK_GBS, 'unit': 'GB/s',
                     'frac': round(achieved / HBM_PEAK_GBS, 4), 'traffic': traffic,
                     'kernel': ('k_sum2_run<DDL_FLOAT, default variant, 4 tiles>' if 32 <= args.bucket_mib < 128 and
                                args.variant < 0 else 'k_sum2_tile<DDL_FLOAT, default variant>'),
                     'kernel_ms': round(kernel_ms, 4),
                     'algorithmic_bytes_per_launch': 3 * S,
                     'frac_of_measured_copy_peak': round(achieved / HBM_MEASURED_GBS, 4)},
    }
    out.update(extra)
    from ddl.torch.communicator import Communicator
    if not args.no_host:
        out['host_resident'] = host_resident_rate(lib, Communicator.world(), S, reps=8)
    if not args.no_fusion:
        del sets
        out['fusion_c5'] = fusion_c5(lib, Communicator.world(), dev, steps=5, forced=not args.no_forced_data_plane)
        if not args.no_host:
            out['keyed_host_c5'] = keyed_host_c5(lib, Communicator.world(), steps=3)
            out['keyed_host_c5_pinned'] = keyed_host_c5(lib, Communicator.world(), steps=3, pinned=True)
            # pageable tensors with the opt-in registration cache: registered on the first batch,
            # then the pinned paths
            out['keyed_host_c5_registered'] = keyed_host_c5(
                lib, Communicator.world(), steps=3, settings={'host_register_cache_bytes': 4 << 30})
            if not args.no_host_steady:  # the pageable path over consecutive steps
                out['keyed_host_c5_steady'] = keyed_host_c5_steady(Communicator.world())
    if not args.no_cpu_baseline:
        out['cpu_baseline'] = cpu_baseline()
        out['cpu_reduce_op_port'] = cpu_reduce_port(64 << 20, args.cpu_seconds)
        out['cpu_reference_path'] = cpu_reference_path()
    emit(out)


def fold_roofline(lib, dev, sh, S, nb=7, order=0, half=False, form=0, nsets=2, chunk_bytes=None):
    """The N-input fold: out = in + 7 received slices over one P=8 chunk (S/8 fp32), the direct
    schedule's reduce; algorithmic bytes (nb + 2) * chunk. order 0: left fold; 1: MPICH's
    pre-fold + pairwise tree (reference_order at P = 8). `half`: the fp16 fold of C4 (inputs
    widened to fp32, one rounding). `form` (config fold_form): 0 the engine's choice (k_sumN_run
    from 4 MiB chunks of 7+ inputs, k_sumN_tile otherwise), 1 the tile form, 2 the run form.
    `nsets` operand sets rotate launch by launch (each set: in, nb inputs, out); `chunk_bytes`
    overrides the chunk size S / 8."""
    import torch
    from ddl.torch.cpp_backend import check
    es = 2 if half else 4
    n = (chunk_bytes or S // 8) // es
    run_form = form == 2 or (form == 0 and n * es >= (4 << 20) and nb + 1 >= 7)
    vec = n * es // 16
    grid = (vec + 1024) // 1024 if run_form else (vec + 128) // 128  # workgroups (rocprof's grid / 128)
    old_form = lib.ddl_get_config(b'fold_form')
    check(lib.ddl_set_config(b'fold_form', form), 'ddl_set_config fold_form')
    sets = [[torch.rand(n, device=dev).to(torch.float16 if half else torch.float32) for _ in range(nb + 2)]
            for _ in range(nsets)]  # in, 7 inputs, out
    P = ctypes.c_void_p * nb
    per_graph = max(20, nsets)

    def run(k):
        b = sets[k % nsets]
        check(lib.ddl_reduce_fold_ordered(b[-1].data_ptr(), b[0].data_ptr(), P(*[t.data_ptr() for t in b[1:-1]]),
                                          nb, n, 19 if half else DT_FLOAT, order, sh), 'ddl_reduce_fold_ordered')
    for k in range(4):
        run(k)
    torch.cuda.synchronize()
    # the launches captured once into a hipGraph and replayed: back-to-back kernels with no host
    # launch between them (a 4 us kernel would otherwise measure the Python launch rate)
    gs = torch.cuda.Stream()
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph, stream=gs):
        sh_g = gs.cuda_stream
        for k in range(per_graph):
            b = sets[k % nsets]
            check(lib.ddl_reduce_fold_ordered(b[-1].data_ptr(), b[0].data_ptr(),
                                              P(*[t.data_ptr() for t in b[1:-1]]), nb, n, 19 if half else DT_FLOAT,
                                              order, sh_g), 'ddl_reduce_fold_ordered (captured)')
    rounds = []
    for _ in range(3):
        with torch.cuda.stream(gs):
            graph.replay()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(gs)
            graph.replay()
            e1.record(gs)
        torch.cuda.synchronize()
        rounds.append(e0.elapsed_time(e1) / per_graph / 1e3)
    best = sum(rounds) / len(rounds)  # the mean of the rounds (not the best)
    del graph, sets
    check(lib.ddl_set_config(b'fold_form', old_form), 'ddl_set_config fold_form')
    byts = (nb + 2) * n * es
    kname = 'k_sumN_run' if run_form else 'k_sumN_tile'
    return {'kernel': f'{kname}<{"DDL_HALF" if half else "DDL_FLOAT"},{nb},order {order}>', 'chunk_bytes': n * es,
            'operand_sets': nsets, 'working_set_bytes': nsets * byts,
            'timing': f'{per_graph} launches captured into a hipGraph, replayed between HIP events on the replay '
                      'stream; mean of 3 rounds',
            'us': round(best * 1e6, 2), 'rounds_us': [round(r * 1e6, 2) for r in rounds], 'grid_workgroups': grid,
            'algorithmic_bytes_per_launch': byts, 'achieved_GBs': round(byts / best / 1e9, 1),
            'frac_of_peak': round(byts / best / 1e9 / HBM_PEAK_GBS, 4),
            'traffic': (pmc_traffic('fold_fp16_P8_C4_chunk') if half else
                        pmc_traffic('fold_fp32_P8_chunk_run' if run_form else 'fold_fp32_P8_chunk'))
            if order == 0 and chunk_bytes is None and nsets == 2 and ((S == 256 << 20 and not half) or
                                                                    (S == 16 << 20 and half)) else
            pmc_traffic('fold_fp16_P8_C4_chunk_hbm') if half and nsets > 2 else None}


def fold_batch_roofline(lib, dev, sh, buckets=64, per_launch=8, bucket_bytes=16 << 20, P=8, form=0):
    """C4's folds as the grouped allreduce launches them: `buckets` fp16 buckets of `bucket_bytes`
    at P ranks -> one chunk of bucket_bytes / P per bucket with P - 1 received inputs; the chunks of
    `per_launch` buckets share one launch (ddl_reduce_fold_batch, FoldBatch: blockIdx.y = bucket).
    All buckets' operands live at once (64 x 9 x 2 MiB = 1.2 GB: HBM, not the Infinity Cache). The
    launches of one pass over the buckets are captured into a hipGraph and replayed between HIP
    events; `us` is the mean per launch over 3 rounds. `form` (config fold_form): 0 the engine's
    choice, 1 the tile form, 2 the run form."""
    import torch
    from ddl.torch.cpp_backend import check
    nb, es = P - 1, 2
    old_form = lib.ddl_get_config(b'fold_form')
    check(lib.ddl_set_config(b'fold_form', form), 'ddl_set_config')
    n = bucket_bytes // P // es
    sets = [[torch.rand(n, device=dev).half() for _ in range(nb + 2)] for _ in range(buckets)]  # in, inputs, out
    V = ctypes.c_void_p
    launches = []
    for k in range(0, buckets, per_launch):
        grp = sets[k:k + per_launch]
        launches.append(((V * len(grp))(*[b[-1].data_ptr() for b in grp]), (V * len(grp))(*[b[0].data_ptr() for b in grp]),
                         (V * (len(grp) * nb))(*[t.data_ptr() for b in grp for t in b[1:-1]]),
                         (ctypes.c_size_t * len(grp))(*[n] * len(grp)), len(grp)))

    def run(stream):
        for outs, as_, ins, ns, c in launches:
            check(lib.ddl_reduce_fold_batch(c, outs, as_, ins, nb, ns, 19, 0, stream), 'ddl_reduce_fold_batch')
    try:
        run(sh)
        torch.cuda.synchronize()
        gs = torch.cuda.Stream()
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph, stream=gs):  # the form is fixed at capture
            run(gs.cuda_stream)
    finally:
        check(lib.ddl_set_config(b'fold_form', old_form), 'ddl_set_config')
    rounds = []
    for _ in range(3):
        with torch.cuda.stream(gs):
            graph.replay()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(gs)
            graph.replay()
            e1.record(gs)
        torch.cuda.synchronize()
        rounds.append(e0.elapsed_time(e1) / len(launches) / 1e3)
    del graph
    t = sum(rounds) / len(rounds)
    byts = (nb + 2) * n * es * per_launch
    return {'kernel': f'k_sumN_tile<DDL_HALF,{nb},order 0> x {per_launch} problems (blockIdx.y)',
            'chunk_bytes': n * es, 'problems_per_launch': per_launch, 'launches_per_pass': len(launches),
            'grid_workgroups': ((n * es // 16 + 128) // 128) * per_launch,
            'timing': f'{len(launches)} launches (all {buckets} buckets) captured into a hipGraph, replayed between HIP '
                      'events on the replay stream; mean of 3 rounds',
            'us': round(t * 1e6, 2), 'rounds_us': [round(r * 1e6, 2) for r in rounds],
            'algorithmic_bytes_per_launch': byts, 'achieved_GBs': round(byts / t / 1e9, 1),
            'frac_of_peak': round(byts / t / 1e9 / HBM_PEAK_GBS, 4),
            'traffic': pmc_traffic('fold_fp16_P8_C4_batch8')}


def half_dtypes(lib, dev, sh, S):
    """acc += in over S bytes of fp16 / bf16 (C4's dtype), 3 rotating sets."""
    import torch
    from ddl.torch.cpp_backend import check
    res = {}
    for name, td, code in (('fp16', torch.float16, 19), ('bf16', torch.bfloat16, 14)):
        n = S // 2
        sets = [(torch.rand(n, device=dev).to(td), torch.rand(n, device=dev).to(td)) for _ in range(NSETS)]

        def run(k):
            a, b = sets[k % NSETS]
            check(lib.ddl_reduce_local(a.data_ptr(), b.data_ptr(), n, code, sh), 'ddl_reduce_local')
        for k in range(3):
            run(k)
        best = float('inf')
        for _ in range(3):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for k in range(12):
                run(k)
            e1.record()
            torch.cuda.synchronize()
            best = min(best, e0.elapsed_time(e1) / 12 / 1e3)
        res[name] = round(3 * S / best / 1e9, 1)
        del sets
    return res


def fusion_c5(lib, comm, dev, steps, k=4096, forced=True):
    """C5: k buckets, byte sizes log-uniform in [4 KiB, 4 MiB] rounded to 256 B,
    dtype fp32/fp16 with p = 0.5, keys grad_%05d submitted in random order, one batch per step
    through the keyed path (negotiation, dtype grouping, plans, pack -> ring -> unpack)."""
    import numpy as np
    import torch
    from ddl.torch.cpp_backend import DONE_FN, check
    rng = np.random.default_rng(5)
    sizes = (np.exp(rng.uniform(np.log(4096), np.log(4 << 20), size=k)).astype(np.int64) // 256) * 256
    order = rng.permutation(k)
    tensors, dts, keys = [], [], []
    for i in order:
        half = rng.random() < 0.5
        n = int(sizes[i]) // (2 if half else 4)
        tensors.append(torch.randn(n, device=dev).to(torch.float16 if half else torch.float32))
        dts.append(19 if half else 1)
        keys.append(f'grad_{i:05d}'.encode())
    total = sum(t.numel() * t.element_size() for t in tensors)
    K = ctypes.c_char_p * k
    V = ctypes.c_void_p * k
    args = (k, K(*keys), V(*[t.data_ptr() for t in tensors]), V(*[t.data_ptr() for t in tensors]),
            (ctypes.c_size_t * k)(*[t.numel() for t in tensors]), (ctypes.c_int * k)(*dts), 0,
            torch.cuda.current_stream(dev).cuda_stream, DONE_FN(), None)  # DONE_FN() = NULL callback

    def step():
        check(lib.ddl_allreduce_submit_batch(comm.id, *args), 'ddl_allreduce_submit_batch')
        check(lib.ddl_wait_all(comm.id), 'ddl_wait_all')

    def timed():
        step()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            step()
        return (time.perf_counter() - t0) / steps

    dt = timed()
    res = {'buckets': k, 'total_bytes': int(total), 'ms': round(dt * 1e3, 3),
           'bucket_GiBs': round(total / GiB / dt, 2),
           'path': 'keyed batch -> token negotiation -> dtype groups -> plans -> pack -> ring -> unpack (in place)',
           'fusion_pipeline_bytes': int(lib.ddl_get_config(b'fusion_pipeline_bytes'))}
    # the same batch with the fusion pipeline off (one pack, one allreduce, one unpack per plan);
    # at one rank both forms run the data plane for real (one_rank_shortcut = 0), where the
    # allreduce itself is the identity and only pack / unpack / host work remain
    keys_set = (b'fusion_pipeline_bytes', b'one_rank_shortcut')
    old = {kk: lib.ddl_get_config(kk) for kk in keys_set}
    try:
        if comm.size == 1:
            res['note'] = 'one-rank world: the engine skips pack/ring/unpack (out = in), so `ms` is host overhead'
        if comm.size == 1 and not forced:
            pass
        else:
            if comm.size == 1:
                check(lib.ddl_set_config(b'one_rank_shortcut', 0), 'ddl_set_config')
                res['data_plane_forced_ms'] = round(timed() * 1e3, 3)
            check(lib.ddl_set_config(b'fusion_pipeline_bytes', 0), 'ddl_set_config')
            key = 'data_plane_forced_unpipelined_ms' if comm.size == 1 else 'unpipelined_ms'
            res[key] = round(timed() * 1e3, 3)
    finally:
        for kk, v in old.items():
            lib.ddl_set_config(kk, v)
    # the fusion gather/scatter kernels on the same buckets (one launch each, device segment table)
    fused = torch.empty(sum((t.numel() * t.element_size() + 255) // 256 * 256 for t in tensors), dtype=torch.uint8,
                        device=dev)
    ptrs = V(*[t.data_ptr() for t in tensors])
    nbytes = (ctypes.c_size_t * k)(*[t.numel() * t.element_size() for t in tensors])
    sh = torch.cuda.current_stream(dev).cuda_stream
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    check(lib.ddl_pack(fused.data_ptr(), ptrs, nbytes, k, sh), 'ddl_pack')
    e0.record()
    for _ in range(steps):
        check(lib.ddl_pack(fused.data_ptr(), ptrs, nbytes, k, sh), 'ddl_pack')
        check(lib.ddl_unpack(ptrs, fused.data_ptr(), nbytes, k, sh), 'ddl_unpack')
    e1.record()
    torch.cuda.synchronize()
    t = e0.elapsed_time(e1) / 1e3 / (2 * steps)
    g, sc = pmc_traffic('pack_c5_gather'), pmc_traffic('pack_c5_scatter')
    res['pack_unpack'] = {'us_per_launch': round(t * 1e6, 1), 'hbm_GBs': round(2 * total / t / 1e9, 1),
                          'algorithmic_bytes_per_launch': 2 * int(total),
                          'traffic': (g + sc) // 2 if g and sc else None}
    return res


def keyed_bucket_stream(lib, comm, dev, steps, buckets=32, bucket_bytes=8 << 20):
    """DDP-style gradient buckets through the keyed path: `buckets` fp32 buckets of
    `bucket_bytes` (256 MiB in all, the C3 size), each submitted by its own call as a backward
    pass would (so each is its own negotiated round), then one wait — with pipeline_rounds 1 (a
    completion thread fires round n's done() while round n+1 negotiates and enqueues) and 0 (each
    round waited for before the next is negotiated)."""
    import torch
    from ddl.torch.cpp_backend import DONE_FN, check
    ts = [torch.randn(bucket_bytes // 4, device=dev) for _ in range(buckets)]
    sh = torch.cuda.current_stream(dev).cuda_stream
    nodone = DONE_FN()

    def step():
        for i, t in enumerate(ts):
            check(lib.ddl_allreduce_submit(comm.id, f'bucket_{i:03d}'.encode(), t.data_ptr(), t.data_ptr(), t.numel(),
                                           1, 0, sh, nodone, None), 'ddl_allreduce_submit')
        check(lib.ddl_wait_all(comm.id), 'ddl_wait_all')

    res = {'buckets': buckets, 'bucket_bytes': bucket_bytes}
    old = lib.ddl_get_config(b'pipeline_rounds')
    sr, cr = ctypes.c_longlong(), ctypes.c_longlong()

    def rounds():  # negotiation rounds of the world's token ring so far (N > 1)
        check(lib.ddl_control_stats(ctypes.byref(sr), ctypes.byref(cr)), 'ddl_control_stats')
        return sr.value + cr.value

    try:
        # both modes warmed up before either is timed: the rounds' sizes differ between the modes,
        # and the first bucket of each new size class tunes the keyed data plane's schedule (a
        # collective timing pass, seconds over slow transports) — inside whichever mode met it
        # first (r06: over sockets the first-timed mode read 3-14x slower for that reason alone)
        for pipelined in (1, 0, 1, 0):
            check(lib.ddl_set_config(b'pipeline_rounds', pipelined), 'ddl_set_config')
            step()
        torch.cuda.synchronize()
        for pipelined in (1, 0):
            check(lib.ddl_set_config(b'pipeline_rounds', pipelined), 'ddl_set_config')
            step()
            torch.cuda.synchronize()
            r0 = rounds()
            t0 = time.perf_counter()
            for _ in range(steps):
                step()
            dt = (time.perf_counter() - t0) / steps
            tag = 'pipelined' if pipelined else 'unpipelined'
            # buckets submitted while a round runs join the next one: fewer, larger rounds when
            # the engine waits for each round
            res[f'{tag}_rounds_per_step'] = round((rounds() - r0) / steps, 2)
            res[f'{tag}_ms'] = round(dt * 1e3, 3)
            res[f'{tag}_algbw_GiBs'] = round(buckets * bucket_bytes / GiB / dt, 2)
    finally:
        lib.ddl_set_config(b'pipeline_rounds', old)
    del ts
    return res


def keyed_c1_latency(lib, comm, dev, reps=200):
    """C1 through the keyed path at this N: one fp32[1024] tensor, x_r = rank, one
    keyed submit + wait per iteration (negotiation over the star, then the allreduce) — the
    reference's per-request latency case (0.73 ms at P = 2 on its CPU+MPI path).
    Reports the median and best round trip and checks the sum."""
    import torch
    from ddl.torch.cpp_backend import DONE_FN, check
    x = torch.full((1024,), float(comm.rank), device=dev)
    y = torch.empty_like(x)
    sh = torch.cuda.current_stream(dev).cuda_stream
    nodone = DONE_FN()
    ts = []
    for i in range(reps + 10):
        t0 = time.perf_counter()
        check(lib.ddl_allreduce_submit(comm.id, b'C1', x.data_ptr(), y.data_ptr(), 1024, 1, 0, sh, nodone, None),
              'ddl_allreduce_submit')
        check(lib.ddl_wait_all(comm.id), 'ddl_wait_all')
        if i >= 10:
            ts.append(time.perf_counter() - t0)
    torch.cuda.synchronize()
    want = comm.size * (comm.size - 1) / 2
    ts.sort()
    return {'elements': 1024, 'dtype': 'f32', 'reps': reps, 'median_us': round(ts[len(ts) // 2] * 1e6, 1),
            'best_us': round(ts[0] * 1e6, 1), 'sum_ok': bool((y == want).all().item()),
            'path': 'keyed submit -> star negotiation -> allreduce in place on the tensor -> done'}


def keyed_host_c5(lib, comm, steps, k=4096, pinned=False, settings=None, warm_steps=6):
    """C5's bucket set as HOST tensors (the reference's deployment: CPU tensors behind the MPI
    buffers) through the keyed path: negotiation, dtype groups, plans, then per plan in chunks
    through pinned slots: host pack -> H2D -> allreduce -> D2H -> host unpack; with pinned tensors
    (`pinned`) the unpack kernel writes the results into them over PCIe instead of D2H + host
    unpack (ddl_allreduce_submit_batch_mem, DDL_MEMORY_HOST). At one rank the data plane is
    forced (one_rank_shortcut = 0). The rate is PCIe-bound (2 x bytes cross the host link); it is
    never `value`."""
    import numpy as np
    import torch
    from ddl.torch.cpp_backend import DONE_FN, MEMORY_HOST, check
    rng = np.random.default_rng(5)
    sizes = (np.exp(rng.uniform(np.log(4096), np.log(4 << 20), size=k)).astype(np.int64) // 256) * 256
    order = rng.permutation(k)
    tensors, dts, keys = [], [], []
    for i in order:
        half = rng.random() < 0.5
        n = int(sizes[i]) // (2 if half else 4)
        t = torch.randn(n).to(torch.float16 if half else torch.float32)
        tensors.append(t.pin_memory() if pinned else t)
        dts.append(19 if half else 1)
        keys.append(f'{"p" if pinned else "h"}grad_{i:05d}'.encode())
    total = sum(t.numel() * t.element_size() for t in tensors)
    K, V = ctypes.c_char_p * k, ctypes.c_void_p * k
    ptrs = V(*[t.data_ptr() for t in tensors])
    args = (k, K(*keys), ptrs, ptrs, (ctypes.c_size_t * k)(*[t.numel() for t in tensors]), (ctypes.c_int * k)(*dts),
            0, MEMORY_HOST, None, DONE_FN(), None)
    settings = dict(settings or {})
    settings['one_rank_shortcut'] = 0
    old = {kk: lib.ddl_get_config(kk.encode()) for kk in settings}
    try:
        for kk, v in settings.items():
            check(lib.ddl_set_config(kk.encode(), v), 'ddl_set_config')

        def step():
            check(lib.ddl_allreduce_submit_batch_mem(comm.id, *args), 'ddl_allreduce_submit_batch_mem')
            check(lib.ddl_wait_all(comm.id), 'ddl_wait_all')
        # warm-up steps, each timed (freshly pinned tensors read slowly for a while on some boxes,
        # DESIGN §7). A FIXED count: every step is a collective, so every rank must run the same
        # number — a time-based loop could leave one rank a step ahead and hang the others
        warm = []
        for _ in range(max(1, warm_steps)):
            t1 = time.perf_counter()
            step()
            warm.append(round((time.perf_counter() - t1) * 1e3, 2))
        plans0 = lib.ddl_get_config(b'host_zero_copy_plans')
        tl_keys = (b'host_pack_us', b'host_wait_us', b'host_unpack_us', b'host_check_us', b'host_plan_us',
                   b'host_coll_us', b'host_d2h_post_us', b'host_unpack_submit_us', b'host_lane_d2h_wait_us',
                   b'host_lane_copy_us', b'host_lane_copy_bytes', b'host_lane_jobs')
        tl0 = [lib.ddl_get_config(kk) for kk in tl_keys]
        cg0 = cgroup_cpu()
        t0 = time.perf_counter()
        for _ in range(steps):
            step()
        dt = (time.perf_counter() - t0) / steps
        cg1 = cgroup_cpu()
        cgroup = None if not cg0 or not cg1 else {
            'quota_cores': cg0['quota_cores'],
            'cpu_cores_busy': round((cg1['usage_usec'] - cg0['usage_usec']) / 1e6 / (dt * steps), 2),
            'throttled_periods_per_step': (cg1['nr_throttled'] - cg0['nr_throttled']) / steps,
            'throttled_ms_per_step': round((cg1['throttled_usec'] - cg0['throttled_usec']) / 1e3 / steps, 2)}
        zero_copy_plans = lib.ddl_get_config(b'host_zero_copy_plans') - plans0
        # the engine thread's timeline per step: packing chunks into the pinned slots, waiting
        # for a slot's DMA / device work, waiting for the unpack lane (staged results are unpacked
        # by their own copy threads while the next chunks are packed, r04); the rest is
        # negotiation, planning and posting
        tl = [(lib.ddl_get_config(kk) - v) / steps / 1e3 for kk, v in zip(tl_keys, tl0)]
        # plan_ms: the allreduce plans' staging loops (pack + slot waits + unpack + posting);
        # outside them: the pinned-output checks (check_ms), and the rest — submission,
        # negotiation, planning, the last chunks' device work after the loop, done() (rest_ms)
        timeline = {'pack_ms': round(tl[0], 3), 'slot_wait_ms': round(tl[1], 3), 'unpack_ms': round(tl[2], 3),
                    'other_ms': round(dt * 1e3 - sum(tl[:3]), 3), 'check_ms': round(tl[3], 3),
                    'plan_ms': round(tl[4], 3), 'rest_ms': round(dt * 1e3 - tl[3] - tl[4], 3),
                    'coll_post_ms': round(tl[5], 3), 'd2h_post_ms': round(tl[6], 3), 'unpack_submit_ms': round(tl[7], 3),
                    **lane_split(tl[8], tl[9], tl[10] * 1e3, tl[11] * 1e3)}
        registered = {'host_registered_bytes': int(lib.ddl_get_config(b'host_registered_bytes')),
                      'host_register_failures': int(lib.ddl_get_config(b'host_register_failures'))}
    finally:
        for kk, v in old.items():
            lib.ddl_set_config(kk.encode(), v)
    path = ('pinned host tensors -> keyed batch -> negotiation -> plans -> pinned chunks (host pack, H2D, '
            'allreduce), unpack kernel writes the results straight into the tensors over PCIe, in place' if pinned else
            'pageable host tensors -> keyed batch -> negotiation -> plans -> pinned chunks (host pack, H2D, '
            'allreduce, D2H, host unpack), in place')
    return {'buckets': k, 'total_bytes': int(total), 'ms': round(dt * 1e3, 3), 'bucket_GiBs': round(total / GiB / dt, 2),
            'pcie_bytes': 2 * int(total), 'host_chunk_bytes': int(lib.ddl_get_config(b'host_chunk_bytes')),
            'host_copy_threads': int(lib.ddl_get_config(b'host_copy_threads')),
            'device_unpack_plans_per_step': zero_copy_plans / steps, 'path': path, 'engine_thread': timeline,
            'warmup_steps_ms': warm, 'cgroup_cpu': cgroup,
            'settings': {kk: v for kk, v in settings.items() if kk != 'one_rank_shortcut'},
            **(registered if 'host_register_cache_bytes' in settings else {})}


LANE_KEYS = (b'host_lane_d2h_wait_us', b'host_lane_copy_us', b'host_lane_copy_bytes', b'host_lane_jobs')


def lane_split(wait_ms, copy_ms, copy_bytes, jobs):
    """The unpack lane's two phases per step, on the lane thread: polling each
    staged chunk's D2H event (lane_d2h_wait_ms: the DMA still running) and the pinned download
    slot -> pageable output memcpy with the copy threads (lane_copy_ms, at lane_copy_GBs). Their
    sum is the lane's busy time; the engine thread's unpack_ms is the part of it it waited for."""
    return {'lane_d2h_wait_ms': round(wait_ms, 3), 'lane_copy_ms': round(copy_ms, 3),
            'lane_copy_bytes': int(copy_bytes), 'lane_jobs': int(jobs),
            'lane_copy_GBs': round(copy_bytes / (copy_ms * 1e-3) / 1e9, 2) if copy_ms > 0 else None}


def keyed_host_c5_steady(comm, steps=10, warm=2, k=4096, budget_s=25.0):
    """The pageable host path in its steady state: C5's bucket set as
    pageable CPU tensors through the keyed host path (the reference's memcpy in / MPI_Allreduce /
    memcpy out, MPIRingTokenCommunication.cc:575-588), `steps` consecutive batches in one process:
      * fresh: a NEW tensor set every step (the old one freed), registration cache off — a loop
        that reduces freshly computed CPU tensors — through the torch mirror
        (allreduce_async_batch: one native completion group for the batch, Handle.wait per tensor);
      * fresh_native: the same sets through the C-ABI directly (no done callback, ddl_wait_all):
        the difference to `fresh` is the mirror's Python (handles, argument arrays, per-tensor waits);
      * fresh_registered: `fresh` with the registration cache on (host_register_cache_bytes):
        every step registers its new pages, the freed ones leave the cache via the torch mirror's
        storage finalizers;
      * reused / reused_registered: ONE tensor set for every step through the torch mirror, cache
        off / on (a DP loop whose CPU gradients keep their storage: registered once, then the
        pinned paths).
    Per step only the submit + wait is timed; building the next set (first touch of 2.45 GB) is
    reported apart. At one rank the data plane is forced (one_rank_shortcut = 0). Median, p90 and
    the last step decide the torch mirror's default."""
    import numpy as np
    import torch
    from ddl.torch.cpp_backend import DONE_FN, MEMORY_HOST, CPPBackend, check
    from ddl.torch.tensor_communicate import allreduce_async_batch
    from ddl.torch.util import ddl_dtype
    lib = CPPBackend.c_api()
    rng = np.random.default_rng(5)
    sizes = (np.exp(rng.uniform(np.log(4096), np.log(4 << 20), size=k)).astype(np.int64) // 256) * 256
    halfs = rng.random(k) < 0.5
    names = [f'sgrad_{i:05d}' for i in range(k)]
    keys = (ctypes.c_char_p * k)(*[n.encode() for n in names])

    def make(seed):
        return [torch.empty(int(sizes[i]) // (2 if halfs[i] else 4),
                            dtype=torch.float16 if halfs[i] else torch.float32).fill_(float((seed + i) % 7))
                for i in range(k)]

    def native_step(ts):  # the C-ABI as a native binding would call it: no Python done()
        ptrs = (ctypes.c_void_p * k)(*[t.data_ptr() for t in ts])
        check(lib.ddl_allreduce_submit_batch_mem(comm.id, k, keys, ptrs, ptrs,
                                                 (ctypes.c_size_t * k)(*[t.numel() for t in ts]),
                                                 (ctypes.c_int * k)(*[ddl_dtype(t) for t in ts]), 0, MEMORY_HOST,
                                                 None, DONE_FN(), None), 'ddl_allreduce_submit_batch_mem')
        check(lib.ddl_wait_all(comm.id), 'ddl_wait_all')

    def mirror_step(ts):
        for h in allreduce_async_batch(ts, names, comm, outputs=ts):
            h.wait()
    total = int(sum(int(s) for s in sizes))
    res = {'buckets': k, 'total_bytes': total, 'steps': steps, 'warm_steps': warm}
    old = {kk: lib.ddl_get_config(kk) for kk in (b'one_rank_shortcut', b'host_register_cache_bytes')}
    modes = (('fresh', True, False, mirror_step), ('fresh_native', True, False, native_step),
             ('fresh_registered', True, True, mirror_step), ('reused', False, False, mirror_step),
             ('reused_registered', False, True, mirror_step))
    try:
        check(lib.ddl_set_config(b'one_rank_shortcut', 0), 'ddl_set_config')
        for mode, fresh, registered, step in modes:
            check(lib.ddl_set_config(b'host_register_cache_bytes', (4 << 30) if registered else 0), 'ddl_set_config')
            ts, alloc, t_start = [], [], time.perf_counter()
            cur, seed = make(0), 0
            for s in range(warm + steps):
                if s and fresh:
                    t1 = time.perf_counter()
                    cur = None  # the old set goes first (its finalizers release cached ranges)
                    cur, seed = make(s), s
                    alloc.append((time.perf_counter() - t1) * 1e3)
                if s == warm:
                    lane0 = [lib.ddl_get_config(kk) for kk in LANE_KEYS]
                t1 = time.perf_counter()
                step(cur)
                dt = (time.perf_counter() - t1) * 1e3
                if s >= warm:
                    ts.append(round(dt, 2))
                if time.perf_counter() - t_start > budget_s and s >= warm + 2:
                    break  # bounded: a slow mode reports the steps it ran
            # one rank: out = in (the data plane ran and left the values intact)
            ok = comm.size != 1 or all(float(cur[i][0]) == float((seed + i) % 7) for i in (0, k // 2, k - 1))
            cur = None
            srt = sorted(ts)
            res[mode] = {'step_ms': ts, 'median_ms': srt[len(srt) // 2],
                         'p90_ms': srt[min(len(srt) - 1, int(0.9 * len(srt)))], 'last_ms': ts[-1],
                         'bucket_GiBs_median': round(total / GiB / (srt[len(srt) // 2] / 1e3), 2),
                         'new_set_ms_median': round(sorted(alloc)[len(alloc) // 2], 1) if alloc else None,
                         'values_ok': ok,
                         'host_registered_bytes_after': int(lib.ddl_get_config(b'host_registered_bytes'))}
            lane = [(lib.ddl_get_config(kk) - v) / len(ts) for kk, v in zip(LANE_KEYS, lane0)]
            res[mode]['engine_thread'] = lane_split(lane[0] / 1e3, lane[1] / 1e3, lane[2], lane[3])
            check(lib.ddl_set_config(b'host_register_cache_bytes', 0), 'ddl_set_config')  # releases every range
    finally:
        for kk, v in old.items():
            lib.ddl_set_config(kk, v)
    res['default_register_cache_bytes'] = int(old[b'host_register_cache_bytes'])
    res['path'] = ('pageable CPU tensors -> keyed batch -> negotiation -> plans -> pinned chunks (host pack, H2D, '
                   'allreduce, D2H or the unpack kernel into registered tensors, host unpack), in place')
    return res


def cgroup_cpu():
    """This process's cgroup (v2) CPU quota in cores and its throttling counters, or None: the GPU
    boxes give a process a CPU share by quota, and the keyed host legs run up to 16 copy threads."""
    try:
        rel = [l.split(':', 2)[2].strip() for l in open('/proc/self/cgroup') if l.startswith('0::')][0]
        base = '/sys/fs/cgroup' + rel
        if not os.path.exists(base + '/cpu.max') and os.path.exists('/sys/fs/cgroup/cpu.max'):
            base = '/sys/fs/cgroup'  # a cgroup namespace: the process's own group is the root
        if os.path.exists(base + '/cpu.max'):  # cgroup v2
            stat = dict(l.split() for l in open(base + '/cpu.stat'))
            quota, period = open(base + '/cpu.max').read().split()
            return {'quota_cores': None if quota == 'max' else round(int(quota) / int(period), 2),
                    'nr_throttled': int(stat.get('nr_throttled', 0)),
                    'throttled_usec': int(stat.get('throttled_usec', 0)), 'usage_usec': int(stat.get('usage_usec', 0))}
        v1 = '/sys/fs/cgroup/cpu'  # cgroup v1 (the process's own cpu controller mount)
        stat = dict(l.split() for l in open(v1 + '/cpu.stat'))
        quota = int(open(v1 + '/cpu.cfs_quota_us').read())
        period = int(open(v1 + '/cpu.cfs_period_us').read())
        return {'quota_cores': None if quota < 0 else round(quota / period, 2),
                'nr_throttled': int(stat.get('nr_throttled', 0)),
                'throttled_usec': int(stat.get('throttled_time', 0)) // 1000,
                'usage_usec': int(open('/sys/fs/cgroup/cpuacct/cpuacct.usage').read()) // 1000}
    except (OSError, IndexError, ValueError):
        return None


def host_resident_rate(lib, comm, S, reps, warm_calls=60):
    """Deployment case: the bucket starts and ends in (pinned) host memory; ddl_allreduce_host
    pipelines H2D -> device ring -> D2H in 32 MiB chunks. PCIe-inclusive rate, never `value`."""
    import torch
    from ddl.torch.cpp_backend import check
    n = S // 4
    src = torch.rand(n, pin_memory=True)
    dst = torch.empty(n, pin_memory=True)
    # warm-up calls, each timed: the pipeline's H2D and D2H ran serialized for its first tens of
    # calls late in the bench (r04 s2: 10.2 ms per call, then 6.2 ms) — the steady rate
    # is the one a training loop sees, the first calls are reported beside it. A FIXED count:
    # ddl_allreduce_host is a collective, so every rank must make the same number of calls
    warm = []
    for _ in range(max(1, warm_calls)):
        t1 = time.perf_counter()
        check(lib.ddl_allreduce_host(comm.id, src.data_ptr(), dst.data_ptr(), n, DT_FLOAT, 0), 'ddl_allreduce_host')
        warm.append(round((time.perf_counter() - t1) * 1e3, 3))
    t0 = time.perf_counter()
    for _ in range(reps):
        check(lib.ddl_allreduce_host(comm.id, src.data_ptr(), dst.data_ptr(), n, DT_FLOAT, 0), 'ddl_allreduce_host')
    dt = (time.perf_counter() - t0) / reps
    return {'bucket_GiBs': round(S / GiB / dt, 2), 'ms': round(dt * 1e3, 3), 'bucket_bytes': S,
            'warmup_calls_ms': warm[:12], 'warmup_last_ms': warm[-3:], 'warmup_calls': len(warm),
            'path': 'pinned host -> H2D -> ring allreduce -> D2H -> pinned host, 32 MiB chunks on 3 streams',
            'pcie_bytes_per_bucket': 2 * S}


def multi_gpu(args):
    import threading

    import torch
    import torch.distributed as dist
    from ddl.torch.communicator import Communicator
    from ddl.torch.cpp_backend import CPPBackend, check
    rank = int(os.environ.get('RANK', 0))
    world = int(os.environ.get('WORLD_SIZE', 1))
    one_gpu = args.rehearse or args.rehearse_rccl  # every rank on cuda:0
    local = 0 if one_gpu else int(os.environ.get('LOCAL_RANK', rank))
    if args.rehearse_rccl:  # before anything initialises RCCL in this process (tests/_mp_gpu_worker.py)
        os.environ.update({'NCCL_HOSTID': f'ddl-bench-host-{rank}-of-{world}', 'NCCL_SOCKET_IFNAME': 'lo',
                           'NCCL_IB_DISABLE': '1'})

    state = {'out': None, 'leg': 'main'}  # rank 0's result so far; the leg in progress

    def hung():
        # a hung collective must not eat the driver's whole scaling run, and must not pass for a
        # good one: once the headline measurement exists, rank 0 prints it with the unfinished
        # leg named in `incomplete`; every rank then exits WATCHDOG_RC.
        # Ranks other than 0 wait a moment first so a launcher that kills the job on the first
        # non-zero exit does not kill rank 0 before its line is out. A hang in teardown, after
        # the complete line was printed, exits WATCHDOG_TEARDOWN_RC.
        sys.stderr.write(f'[bench rank {rank}] watchdog: leg {state["leg"]!r} not done after '
                         f'{args.watchdog_s:.0f} s, aborting\n')
        sys.stderr.flush()
        if state.get('printed'):
            os._exit(WATCHDOG_TEARDOWN_RC)
        if state['out'] is not None and rank == 0:
            state['out']['incomplete'] = f'watchdog after {args.watchdog_s:.0f} s in leg {state["leg"]}'
            emit(state['out'])
        if rank != 0:
            time.sleep(3.0)
        os._exit(WATCHDOG_RC)

    dog = threading.Timer(args.watchdog_s, hung)
    dog.daemon = True
    dog.start()
    if os.environ.get('DDL_BENCH_WATCHDOG_SELFTEST') == '1':
        _watchdog_selftest(args, state, rank, world)  # never returns: the watchdog ends the process
    if not one_gpu and torch.cuda.device_count() < world:  # counting does not initialise the GPU
        sys.stderr.write(f'[bench rank {rank}] {world} ranks need {world} GPUs, this box has '
                         f'{torch.cuda.device_count()} (use --rehearse to run the N>1 legs on one GPU)\n')
        sys.exit(2)
    torch.cuda.set_device(local)
    os.environ.setdefault('MASTER_ADDR', '127.0.0.1')
    os.environ.setdefault('MASTER_PORT', '29533')
    dist.init_process_group('gloo', rank=rank, world_size=world)
    lib = CPPBackend.c_api()
    if args.rehearse:  # every rank on cuda:0, groups over gloo (--rehearse-rccl: real RCCL over sockets)
        sys.path.insert(0, os.path.join(ROOT, 'tools'))
        import gloo_transport
        state['callbacks'] = gloo_transport.init_world(lib, dist, torch, rank, world, device=local)
    elif args.rehearse_rccl:  # the product's bootstrap on cuda:0 (init reads LOCAL_RANK otherwise)
        from ddl.torch.communicator import init as ddl_world_init
        ddl_world_init(rank, world, 0)
    comm = Communicator.world()
    kind, tranks = ctypes.c_int(), ctypes.c_int()
    check(lib.ddl_comm_transport(comm.id, ctypes.byref(kind), ctypes.byref(tranks)), 'ddl_comm_transport')
    transport = {'kind': ('none', 'rccl', 'test_transport_gloo')[kind.value], 'ranks': tranks.value,
                 'rccl_ranks': tranks.value if kind.value == 1 else None}
    if tranks.value != world:
        sys.stderr.write(f'[bench rank {rank}] the transport sees {tranks.value} ranks, the launcher {world}\n')
        sys.exit(2)
    # which executor and transport each leg's collectives ran on
    executor_path = ('RingExecutor::run_ over ' + {'rccl': 'RcclTransport (ncclSend/ncclRecv groups, ncclAllGather)',
                                                     'test_transport_gloo': 'CallbackTransport (gloo host copies)',
                                                     'none': 'no transport (one rank)'}[transport['kind']])
    keyed_path = ('RequestHandler (star negotiation over TCP) -> FusionPipe -> the private keyed communicator\'s '
                  + executor_path)
    dev = torch.device('cuda', local)
    S = args.bucket_mib << 20
    n = S // 4
    g = torch.Generator(device=dev).manual_seed(1234 + 7919 * rank)
    send = torch.randn(n, device=dev, generator=g)
    recv = torch.empty_like(send)
    stream = torch.cuda.current_stream(dev)

    def step(variant=0):
        check(lib.ddl_allreduce_variant(comm.id, send.data_ptr(), recv.data_ptr(), n, DT_FLOAT, 0,
                                        stream.cuda_stream, variant), 'ddl_allreduce_variant')

    def timed_fn(fn, steps, warmup):
        for _ in range(warmup):
            fn()
        torch.cuda.synchronize()
        dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            fn()
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        dist.barrier()
        t = torch.tensor([el], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return t.item() / steps

    def timed(variant, steps, warmup):
        return timed_fn(lambda: step(variant), steps, warmup)

    sec = timed(0, args.steps, args.warmup)
    # reduce-kernel roofline: time every reduce launch on the engine's compute stream
    check(lib.ddl_kernel_timing(comm.id, 1), 'ddl_kernel_timing')
    for _ in range(min(args.steps, 10)):
        step(0)
    torch.cuda.synchronize()
    check(lib.ddl_kernel_timing(comm.id, 0), 'ddl_kernel_timing')
    launches, kbytes, kms = ctypes.c_longlong(), ctypes.c_double(), ctypes.c_double()
    check(lib.ddl_kernel_stats(comm.id, ctypes.byref(launches), ctypes.byref(kbytes), ctypes.byref(kms)),
          'ddl_kernel_stats')
    # the autotuner's record for this bucket (tuned during the first warmup call)
    tune = None
    chosen, count = ctypes.c_int(-1), ctypes.c_int(0)
    cfgs = (ctypes.c_longlong * 128)()
    tms = (ctypes.c_float * 32)()
    check(lib.ddl_tune_result(comm.id, S, ctypes.byref(chosen), ctypes.byref(count), cfgs, tms, 32),
          'ddl_tune_result')
    if chosen.value >= 0:
        tune = tuner_table(chosen, count, cfgs, tms)
    # correctness spot check: every rank's sum must match (checksum of checksums)
    step(0)
    torch.cuda.synchronize()
    cs = torch.tensor([recv.double().sum().item()], dtype=torch.float64)
    ref = torch.tensor([send.double().sum().item()], dtype=torch.float64)
    dist.all_reduce(ref)
    cs_max, cs_min = cs.clone(), cs.clone()
    dist.all_reduce(cs_max, op=dist.ReduceOp.MAX)
    dist.all_reduce(cs_min, op=dist.ReduceOp.MIN)

    ms = sec * 1e3
    algbw = S / GiB / sec
    busbw_gbs = 2 * (world - 1) / world * S / sec / 1e9
    ceiling = link_ceiling(world)
    avg_kernel_ms = kms.value / max(1, launches.value)
    achieved = kbytes.value / max(1e-9, kms.value / 1e3) / 1e9
    out = {
        'metric': 'device-resident allreduce GiB/s vs bucket size at 1/2/4/8 MI355X',
        'value': round(algbw, 2),
        'unit': 'GiB/s',
        'n_gpus': world,
        'steps': args.steps,
        'warmup': args.warmup,
        'ms_per_step': round(ms, 4),
        'higher_is_better': True,
        'scaling': 'weak',
        'vs_baseline': None,
        'dtype': 'f32',
        'data': 'synthetic N(0,1) fp32 bucket per rank, resident in HBM',
        'config': {'workload': f'C3: allreduce (autotuned RS+AG schedule over RCCL send/recv, HIP reduce; '
                               f'sums in MPICH MPI_Allreduce order, bit-equal to the reference), fp32 '
                               f'{args.bucket_mib} MiB bucket per rank, {world}xMI355X',
                   'bucket_bytes': S, 'parallelism': f'dp{world}',
                   'reference_order': lib.ddl_get_config(b'reference_order')},
        'value_is': 'allreduce algbw: bucket bytes / max-over-ranks time per allreduce (GiB/s)',
        'transport': transport,
        'legs_path': {'headline, parity, schedule_sweep, c4, size_sweep, broadcast_allgather': executor_path,
                      'host_resident': 'ddl_allreduce_host: H2D / D2H chunks around ' + executor_path,
                      'fusion_c5, keyed_bucket_stream, keyed_c1_latency, keyed_host_c5_pinned': keyed_path,
                      'rccl_allreduce_comparator': "RCCL's own ncclAllReduce on the world's communicator",
                      'compute_cu_mask_ab': 'a split communicator: ' + executor_path},
        'algbw_GiBs': round(algbw, 2),
        'busbw_GBs': round(busbw_gbs, 2),
        'link_roofline': (None if ceiling is None else
                          dict(ceiling, frac=round(busbw_gbs / ceiling['busbw_ceiling_GBs'], 4),
                               algbw_frac=round(algbw * GiB / 1e9 / ceiling['algbw_ceiling_GBs'], 4))),
        'autotune': tune,
        'roofline': {'bound': 'hbm', 'achieved': round(achieved, 1), 'peak': HBM_PEAK_GBS, 'unit': 'GB/s',
                     'frac': round(achieved / HBM_PEAK_GBS, 4), 'traffic': None,
                     'traffic_note': 'no PMC pass on the node; the same kernels measured 1.0001-1.0002x '
                                     'algorithmic bytes on one GPU (profiles/pmc_traffic.json)',
                     'kernel': (f'k_sumN_run / k_sumN_tile<float,{world - 1}> ({tune["chosen"]["algo"]} fold; run form '
                                f'from 4 MiB slices at P >= 7)'
                                if tune and tune['chosen']['algo'] != 'ring' else
                                'k_sum2_tile<float> (reduce-scatter step, all rings in one launch)'),
                     'avg_kernel_ms': round(avg_kernel_ms, 4), 'launches_timed': launches.value},
        'check': {'sum_of_recv_min': cs_min.item(), 'sum_of_recv_max': cs_max.item(),
                  'sum_of_inputs': ref.item()},
    }
    if args.rehearse:
        out['rehearsal'] = 'point-to-point over gloo host copies on one GPU: exercises the N>1 legs, NOT a measurement'
    elif args.rehearse_rccl:
        out['rehearsal'] = ('real multi-rank RCCL communicators on one GPU (NCCL_HOSTID per rank: RCCL\'s socket '
                            'transport over loopback): the node\'s code path end to end, NOT an xGMI measurement')
    state['out'] = out  # from here on a hung optional leg still reports the headline result
    # parity on this node first, so no optional leg can hide it: every rank's result equals
    # MPI_Allreduce's (MPICH 3.3.2 order) bit for bit, on both sides of MPICH's 2048-byte switch
    state['leg'] = 'parity'
    try:
        out['parity_vs_mpich_order'] = parity_leg(lib, comm, dist, torch, dev, stream, rank, world)
    except Exception as e:
        out['parity_vs_mpich_order'] = {'bit_exact': False, 'error': repr(e)[:400]}

    # the reference's own CPU+MPI path at this N, on the host cores: rank 0
    # runs oracle/ref_path_port.c under MPICH at P = N on the C3 shape (cpu_baseline) and the C1 /
    # C3 / C5-like legs (cpu_reference_path) while the other ranks wait at the barrier — no GPU
    # work runs meanwhile. Right after the parity leg, so a later optional leg that hangs (the
    # watchdog then prints the line as it stands) cannot cost the line its baseline. Path restated:
    # RingTokenCommunicateHandler.cc:327-410 -> MPIRingTokenCommunication.cc:548-733 ->
    # MPICommunicator.cc:14-28.
    state['leg'] = 'cpu_baseline'
    dist.barrier()
    if rank == 0 and not args.no_cpu_baseline:
        try:
            out['cpu_baseline'] = cpu_baseline(P=world, reps=4)
            out['cpu_reference_path'] = cpu_reference_path()
        except Exception as e:  # a failed optional leg must not cost the headline line
            out.setdefault('leg_errors', {})['cpu_baseline'] = repr(e)[:400]
    dist.barrier()
    state['leg'] = 'rccl_comparator'
    try:
        if not args.rehearse:
            sec_rccl = timed(1, max(5, args.steps // 2), 3)
            out['rccl_allreduce_comparator'] = {'ms': round(sec_rccl * 1e3, 4),
                                                'busbw_GBs': round(2 * (world - 1) / world * S / sec_rccl / 1e9, 2)}
    except Exception as e:  # a failed optional leg must not cost the headline line
        out.setdefault('leg_errors', {})['rccl_comparator'] = repr(e)[:400]
    # CUs left to RCCL (config compute_cu_mask): the same allreduce on a communicator
    # whose executor's compute stream avoids every 8th CU, beside the world's (all CUs); the mask is
    # read when an executor is created, so a split over every rank carries it
    state['leg'] = 'compute_cu_mask_ab'
    try:
        if True:  # (rehearsed too: the split and the masked executor run; the times mean nothing there)
            check(lib.ddl_set_config(b'compute_cu_mask', 8), 'ddl_set_config')
            sub = comm.split_communicator(0, rank)
            check(lib.ddl_set_config(b'compute_cu_mask', 0), 'ddl_set_config')

            def sub_step():
                check(lib.ddl_allreduce(sub.id, send.data_ptr(), recv.data_ptr(), n, DT_FLOAT, 0, stream.cuda_stream),
                      'ddl_allreduce (masked)')
            reps = max(5, args.steps // 2)
            t_masked = timed_fn(sub_step, reps, 3)  # the first warmup call tunes the new communicator
            t_world = timed_fn(lambda: step(0), reps, 3)
            out['compute_cu_mask_ab'] = {'every_8th_cu_off_ms': round(t_masked * 1e3, 4),
                                         'all_cus_ms': round(t_world * 1e3, 4),
                                         'speedup_masked': round(t_world / t_masked, 4)}
            sub.detach()
    except Exception as e:  # a failed optional leg must not cost the headline line
        out.setdefault('leg_errors', {})['compute_cu_mask_ab'] = repr(e)[:400]
    # RCCL channel (CTA) bounds (config rccl_min_ctas / rccl_max_ctas = ncclConfig_t.minCTAs /
    # maxCTAs): the headline allreduce on a split communicator created under
    # each setting, beside the world's (RCCL's own channel count). Whether the direct schedule's
    # P-1 concurrent sends / receives fill P-1 xGMI links depends on the p2p channels RCCL gives
    # them, which these bounds cap; DESIGN §8 reads the default off this field. Every rank sets
    # the same values in the same order (shared tunables).
    # The tuner is off for the whole leg (every rank alike), so the world and each split run the
    # same configured schedule and only the channel bounds differ.
    state['leg'] = 'rccl_cta_sweep'
    tune_before = lib.ddl_get_config(b'tune')
    try:
        if not args.no_cta_sweep:
            check(lib.ddl_set_config(b'tune', 0), 'ddl_set_config')
            cta = []
            reps = max(5, args.steps // 2)
            t_world = timed_fn(lambda: step(0), reps, 3)
            for lo, hi in ((8, 8), (16, 16), (32, 32), (64, 64)):
                check(lib.ddl_set_config(b'rccl_min_ctas', lo), 'ddl_set_config')
                check(lib.ddl_set_config(b'rccl_max_ctas', hi), 'ddl_set_config')
                try:
                    sub = comm.split_communicator(0, rank)
                finally:
                    check(lib.ddl_set_config(b'rccl_min_ctas', 0), 'ddl_set_config')
                    check(lib.ddl_set_config(b'rccl_max_ctas', 0), 'ddl_set_config')

                def sub_step(sub=sub):
                    check(lib.ddl_allreduce(sub.id, send.data_ptr(), recv.data_ptr(), n, DT_FLOAT, 0,
                                            stream.cuda_stream), 'ddl_allreduce (cta split)')
                t = timed_fn(sub_step, reps, 3)  # the first warmup call agrees the config on the split
                cta.append({'min_ctas': lo, 'max_ctas': hi, 'ms': round(t * 1e3, 4),
                            'busbw_GBs': round(2 * (world - 1) / world * S / t / 1e9, 2),
                            'speedup_vs_default': round(t_world / t, 4)})
                sub.detach()
                out['rccl_cta_sweep'] = {'default_ms': round(t_world * 1e3, 4), 'bucket_bytes': S, 'tune': 0,
                                         'settings': cta}
    except Exception as e:  # a failed optional leg must not cost the headline line
        out.setdefault('leg_errors', {})['rccl_cta_sweep'] = repr(e)[:400]
    finally:
        lib.ddl_set_config(b'tune', tune_before)
    # fixed schedules, tuner off (every rank sets the same values in the same order: the
    # schedule must be identical on all ranks)
    state['leg'] = 'schedule_sweep'
    try:
        sweep = []
        if not args.no_config_sweep:
            keys = ('algo', 'rings', 'slice_bytes', 'tune', 'reference_order')
            defaults = {k: lib.ddl_get_config(k.encode()) for k in keys}
            lib.ddl_set_config(b'tune', 0)
            # each schedule as such (with reference_order a ring at P > 2 would run as direct)
            lib.ddl_set_config(b'reference_order', 0)
            try:
                for algo, rings, slice_mib in ((0, 8, 2), (0, 1, 2), (0, 8, 1), (0, 8, 4), (0, 8, 8), (0, 3, 2),
                                               (0, 8, 64), (1, 1, 2), (1, 1, 8), (1, 1, 64), (4, 1, 2), (4, 1, 8),
                                               (4, 1, 64)):
                    if algo in (1, 4) and world < 3:
                        continue
                    lib.ddl_set_config(b'algo', algo)
                    lib.ddl_set_config(b'rings', rings)
                    lib.ddl_set_config(b'slice_bytes', slice_mib << 20)
                    t = timed(0, max(5, args.steps // 4), 2)
                    sweep.append({'algo': algo_name(algo), 'rings': rings, 'slice_MiB': slice_mib,
                                  'ms': round(t * 1e3, 4),
                                  'busbw_GBs': round(2 * (world - 1) / world * S / t / 1e9, 2)})
                    out['schedule_sweep'] = sweep
            finally:  # every rank restores the same shared config
                for k, v in defaults.items():
                    lib.ddl_set_config(k.encode(), v)
    except Exception as e:  # a failed optional leg must not cost the headline line
        out.setdefault('leg_errors', {})['schedule_sweep'] = repr(e)[:400]
    # C4: fp16, 1 GiB as 64 x 16 MiB buckets, one ddl_allreduce per bucket
    state['leg'] = 'c4'
    try:
        if not args.no_c4:
            nb = (16 << 20) // 2
            c4_bufs = [torch.randn(nb, device=dev, generator=g).half() for _ in range(64)]

            def c4_step():
                for b in c4_bufs:
                    check(lib.ddl_allreduce(comm.id, b.data_ptr(), b.data_ptr(), nb, 19, 0, stream.cuda_stream),
                          'ddl_allreduce')
            t = timed_fn(c4_step, 3, 1)
            out['c4_fp16_64x16MiB'] = {'buckets': 64, 'bucket_bytes': 16 << 20, 'ms': round(t * 1e3, 3),
                                       'algbw_GiBs': round((1 << 30) / GiB / t, 2),
                                       'busbw_GBs': round(2 * (world - 1) / world * (1 << 30) / t / 1e9, 2),
                                       'path': 'one ddl_allreduce per bucket: ' + executor_path}
            # the tuner's table for the 16 MiB class (its candidates include 4 and 8 slices per
            # chunk, so a slice's fold can run under the next slice's reduce-scatter)
            c4_chosen, c4_count = ctypes.c_int(-1), ctypes.c_int(0)
            check(lib.ddl_tune_result(comm.id, 16 << 20, ctypes.byref(c4_chosen), ctypes.byref(c4_count), cfgs, tms,
                                      32), 'ddl_tune_result')
            if c4_chosen.value >= 0:
                out['c4_fp16_64x16MiB']['tuner'] = tuner_table(c4_chosen, c4_count, cfgs, tms)
            # the same 64 buckets as ONE grouped call (ddl_allreduce_batch): one RCCL group per tick for
            # every bucket, the folds of 8 buckets per launch; bit-identical sums
            V = ctypes.c_void_p * 64
            ptrs = V(*[b.data_ptr() for b in c4_bufs])
            counts = (ctypes.c_size_t * 64)(*[nb] * 64)

            def c4_batch_step():
                check(lib.ddl_allreduce_batch(comm.id, 64, ptrs, ptrs, counts, 19, 0, stream.cuda_stream),
                      'ddl_allreduce_batch')
            t = timed_fn(c4_batch_step, 3, 1)
            out['c4_fp16_64x16MiB_batch'] = {'buckets': 64, 'bucket_bytes': 16 << 20, 'ms': round(t * 1e3, 3),
                                             'algbw_GiBs': round((1 << 30) / GiB / t, 2),
                                             'busbw_GBs': round(2 * (world - 1) / world * (1 << 30) / t / 1e9, 2),
                                             'path': 'one ddl_allreduce_batch of 64 buckets: ' + executor_path}
            del c4_bufs
    except Exception as e:  # a failed optional leg must not cost the headline line
        out.setdefault('leg_errors', {})['c4'] = repr(e)[:400]
    # broadcast (root 0) and allgather of the same bucket size (§8f #3)
    state['leg'] = 'broadcast_allgather'
    try:
        if not args.no_collectives:
            bc = recv.clone()
            t_b = timed_fn(lambda: check(lib.ddl_broadcast(comm.id, bc.data_ptr(), n, DT_FLOAT, 0, stream.cuda_stream),
                                         'ddl_broadcast'), max(5, args.steps // 4), 2)
            per = n // world
            t_g = timed_fn(lambda: check(lib.ddl_allgather(comm.id, send.data_ptr(), per, recv.data_ptr(), per, DT_FLOAT,
                                                           stream.cuda_stream), 'ddl_allgather'),
                           max(5, args.steps // 4), 2)
            out['broadcast_allgather'] = {
                'broadcast': {'bytes': S, 'ms': round(t_b * 1e3, 4), 'algbw_GiBs': round(S / GiB / t_b, 2),
                              'root_link_bytes': 2 * S // world},
                'allgather': {'bytes_out': per * world * 4, 'ms': round(t_g * 1e3, 4),
                              'algbw_GiBs': round(per * world * 4 / GiB / t_g, 2),
                              'busbw_GBs': round((world - 1) * per * 4 / t_g / 1e9, 2)}}
            del bc
    except Exception as e:  # a failed optional leg must not cost the headline line
        out.setdefault('leg_errors', {})['broadcast_allgather'] = repr(e)[:400]
    state['leg'] = 'host_resident'
    try:
        if not args.no_host:
            out['host_resident'] = host_resident_rate(lib, comm, S, reps=4, warm_calls=1 if one_gpu else 20)
    except Exception as e:  # a failed optional leg must not cost the headline line
        out.setdefault('leg_errors', {})['host_resident'] = repr(e)[:400]
    state['leg'] = 'fusion_c5'
    try:
        if not args.no_fusion:
            out['fusion_c5'] = fusion_c5(lib, comm, dev, steps=3)
    except Exception as e:  # a failed optional leg must not cost the headline line
        out.setdefault('leg_errors', {})['fusion_c5'] = repr(e)[:400]
    state['leg'] = 'keyed_bucket_stream'
    try:
        if not args.no_fusion:
            out['keyed_bucket_stream'] = keyed_bucket_stream(lib, comm, dev, steps=3)
    except Exception as e:  # a failed optional leg must not cost the headline line
        out.setdefault('leg_errors', {})['keyed_bucket_stream'] = repr(e)[:400]
    state['leg'] = 'keyed_c1_latency'
    try:
        out['keyed_c1_latency'] = keyed_c1_latency(lib, comm, dev)
    except Exception as e:  # a failed optional leg must not cost the headline line
        out.setdefault('leg_errors', {})['keyed_c1_latency'] = repr(e)[:400]
    # the deployment case at N ranks: C5's buckets as pinned host tensors through the keyed path
    # (host pack -> H2D -> allreduce over xGMI -> unpack kernel into the tensors over PCIe)
    state['leg'] = 'keyed_host_c5_pinned'
    try:
        if not args.no_fusion and not args.no_host:
            out['keyed_host_c5_pinned'] = keyed_host_c5(lib, comm, steps=2, pinned=True,
                                                        warm_steps=1 if one_gpu else 3)
    except Exception as e:  # a failed optional leg must not cost the headline line
        out.setdefault('leg_errors', {})['keyed_host_c5_pinned'] = repr(e)[:400]
    # the metric's curve: allreduce GiB/s vs bucket size at this N, the engine (autotuned per
    # size class) next to RCCL's own ncclAllReduce on the same buffers
    state['leg'] = 'size_sweep'
    try:
        if not args.no_size_sweep:
            curve = []
            for sz in [(4 << 10) << (2 * k) for k in range(10)]:  # 4 KiB, 16 KiB, ..., 1 GiB
                if sz > args.size_sweep_max_mib << 20:
                    break
                m = sz // 4
                a = torch.randn(m, device=dev, generator=g)
                b = torch.empty_like(a)
                reps = int(min(200, max(5, (64 << 20) // sz)))

                def one(variant, a=a, b=b, m=m):
                    check(lib.ddl_allreduce_variant(comm.id, a.data_ptr(), b.data_ptr(), m, DT_FLOAT, 0,
                                                    stream.cuda_stream, variant), 'ddl_allreduce_variant')
                t_ours = timed_fn(lambda: one(0), reps, 3)
                t_rccl = t_ours if args.rehearse else timed_fn(lambda: one(1), reps, 3)
                chosen, count = ctypes.c_int(-1), ctypes.c_int(0)
                check(lib.ddl_tune_result(comm.id, sz, ctypes.byref(chosen), ctypes.byref(count), cfgs, tms, 32),
                      'ddl_tune_result')
                pick = None
                if chosen.value >= 0:
                    i = chosen.value
                    pick = f"{algo_name(cfgs[4 * i])}/r{cfgs[4 * i + 1]}/s{cfgs[4 * i + 2] >> 10}K"
                curve.append({'bytes': sz, 'us': round(t_ours * 1e6, 1), 'algbw_GiBs': round(sz / GiB / t_ours, 3),
                              'busbw_GBs': round(2 * (world - 1) / world * sz / t_ours / 1e9, 2),
                              'rccl_us': round(t_rccl * 1e6, 1),
                              'rccl_busbw_GBs': round(2 * (world - 1) / world * sz / t_rccl / 1e9, 2),
                              'schedule': pick})
                out['size_sweep_fp32'] = curve
                del a, b
    except Exception as e:  # a failed optional leg must not cost the headline line
        out.setdefault('leg_errors', {})['size_sweep'] = repr(e)[:400]
    # the latency-bound end of the curve again with the allreduces captured into a hipGraph
    # (each size class was tuned above, outside the capture): no host enqueue per call
    state['leg'] = 'size_sweep_graph'
    try:
        if not args.no_size_sweep:
            gcurve = []
            for sz in [(4 << 10) << (2 * k) for k in range(6)]:  # 4 KiB .. 4 MiB
                if sz > args.size_sweep_max_mib << 20:
                    break
                m = sz // 4
                a = torch.full((m,), float(rank + 1), device=dev)  # the replayed sums are checkable
                b = torch.empty_like(a)
                per_graph, replays = 16, 10
                gs = torch.cuda.Stream()
                with torch.cuda.stream(gs):  # warm: tuned class, staging and events sized
                    check(lib.ddl_allreduce(comm.id, a.data_ptr(), b.data_ptr(), m, DT_FLOAT, 0, gs.cuda_stream),
                          'ddl_allreduce')
                torch.cuda.synchronize()
                graph = torch.cuda.CUDAGraph()
                with torch.cuda.graph(graph, stream=gs):
                    for _ in range(per_graph):
                        check(lib.ddl_allreduce(comm.id, a.data_ptr(), b.data_ptr(), m, DT_FLOAT, 0, gs.cuda_stream),
                              'ddl_allreduce (captured)')

                def replay(graph=graph, gs=gs):
                    with torch.cuda.stream(gs):
                        graph.replay()
                b.fill_(-1.0)
                torch.cuda.synchronize()
                t = timed_fn(replay, replays, 1) / per_graph
                torch.cuda.synchronize()
                ok = torch.tensor([int(bool((b == float(world * (world + 1) // 2)).all().item()))])
                dist.all_reduce(ok, op=dist.ReduceOp.MIN)  # every rank's replayed sums exact
                gcurve.append({'bytes': sz, 'us': round(t * 1e6, 1), 'algbw_GiBs': round(sz / GiB / t, 3),
                               'busbw_GBs': round(2 * (world - 1) / world * sz / t / 1e9, 2),
                               'replay_exact': bool(ok.item())})
                out['size_sweep_graph_fp32'] = gcurve
                # every captured graph must be gone before finalize: RCCL keeps a captured
                # collective's resources until its graph is destroyed, and ncclCommDestroy waits for
                # them (r06 s18: the replay closure kept the last graph alive and teardown hung)
                del graph, a, b, replay
    except Exception as e:  # e.g. the rehearsal's host-synchronising transport cannot be captured
        out.setdefault('leg_errors', {})['size_sweep_graph'] = repr(e)[:400]
    finally:  # also after a failed capture: no graph may outlive this leg
        import gc
        graph = replay = None
        gc.collect()
        torch.cuda.synchronize()
    state['leg'] = 'finalize'
    if rank == 0:
        emit(out)
    state['printed'] = True  # a hang in teardown must not print a second line
    dist.barrier()
    from ddl.torch.communicator import finalize
    finalize()
    dist.destroy_process_group()
    dog.cancel()


def tuner_table(chosen, count, cfgs, tms):
    """ddl_tune_result's record as {'chosen', 'candidates'} (slice_KiB per chunk slice)."""
    cands = [{'algo': algo_name(cfgs[4 * i]), 'rings': cfgs[4 * i + 1], 'slice_KiB': cfgs[4 * i + 2] >> 10,
              'max_slices': cfgs[4 * i + 3], 'ms': round(tms[i], 4)} for i in range(min(count.value, 32))]
    return {'chosen': cands[chosen.value], 'candidates': cands}


ALGO_NAMES = ('ring', 'direct', 'oneshot', 'gatherfold', 'direct_gather')  # schedule.h enum Algo


def algo_name(a):
    return ALGO_NAMES[a] if 0 <= a < len(ALGO_NAMES) else f'algo{a}'


def link_ceiling(P, S=None):
    """Roofline of one allreduce at P ranks, in busbw = 2(P-1)/P x S / t terms.
    The reference-order direct schedule (what runs at P > 2): each rank sends chunk-slices to its
    P-1 peers at once in the reduce-scatter and again in the allgather, so each of its P-1 xGMI
    links carries 2S/P per allreduce -> t >= 2S / (P x B_link), busbw <= (P-1) x B_link (the
    same as P-1 edge-disjoint rings). HBM per rank: (5P-3)/P x S bytes (RS send reads + staging
    writes, the fold's P inputs + 1 output, AG send reads + receive writes) -> busbw <=
    2(P-1)/(5P-3) x HBM. The ceiling is the smaller. None at P = 1 (no exchange)."""
    if P < 2:
        return None
    links = (P - 1) * XGMI_LINK_GBS
    hbm = 2 * (P - 1) / (5 * P - 3) * HBM_PEAK_GBS
    bus = min(links, hbm)
    return {'bound': 'xgmi' if links <= hbm else 'hbm', 'busbw_ceiling_GBs': round(bus, 1),
            'algbw_ceiling_GBs': round(bus * P / (2 * (P - 1)), 1), 'link_GBs': XGMI_LINK_GBS,
            'links_used': P - 1, 'hbm_term_GBs': round(hbm, 1),
            'formula': 'busbw <= min((P-1) x B_link, 2(P-1)/(5P-3) x HBM)'}


def mpich_order_sum(xs, message_bytes):
    """MPI_Allreduce(MPI_SUM)'s per-element order in MPICH 3.3.2 (numpy, one rounding per add in
    the element type): a binomial tree over ranks up to 2048 bytes (or when the element count is
    below pof2), else the first 2*rem ranks folded in pairs and a pairwise tree over the pof2
    leaves. A check of the N>1 run only; the tests pin the same order against MPICH itself
    (tests/test_live_mpich.py)."""
    v = [x.copy() for x in xs]
    k = len(v)
    pof2 = 1
    while pof2 * 2 <= k:
        pof2 *= 2
    if message_bytes <= 2048 or message_bytes // xs[0].itemsize < pof2:
        m = 1
        while m < k:
            for t in range(0, k - m, 2 * m):
                v[t] = v[t] + v[t + m]
            m *= 2
        return v[0]
    rem = k - pof2
    leaf = [v[2 * t] + v[2 * t + 1] for t in range(rem)] + v[2 * rem:]
    m = 1
    while m < pof2:
        for t in range(0, pof2, 2 * m):
            leaf[t] = leaf[t] + leaf[t + m]
        m *= 2
    return leaf[0]


def parity_leg(lib, comm, dist, torch, dev, stream, rank, world):
    """ddl_allreduce (the engine's default: autotuned, reference order) of seeded buckets; the
    inputs and every rank's output are gathered on rank 0 over gloo and compared with MPICH's
    order. Returns {case: bit_exact} and the overall verdict."""
    import numpy as np
    from ddl.torch.cpp_backend import check
    cases = [('fp32_300', DT_FLOAT, np.float32, 300), ('fp32_1Mi+3', DT_FLOAT, np.float32, (1 << 20) + 3),
             ('fp64_257', 2, np.float64, 257), ('int32_4099', 3, np.int32, 4099)]
    res = {}
    for name, dt, npt, n in cases:
        rng = np.random.default_rng(99 + 7919 * rank + n)
        x = (rng.integers(-2 ** 31, 2 ** 31, n, dtype=np.int64).astype(np.int32) if npt is np.int32
             else rng.standard_normal(n).astype(npt))
        t = torch.from_numpy(x.copy()).to(dev)
        check(lib.ddl_allreduce(comm.id, t.data_ptr(), t.data_ptr(), n, dt, 0, stream.cuda_stream), 'ddl_allreduce')
        torch.cuda.synchronize()
        mine = torch.from_numpy(np.stack([x, t.cpu().numpy()]))
        everyone = [torch.empty_like(mine) for _ in range(world)]
        dist.all_gather(everyone, mine)
        if rank == 0:
            want = mpich_order_sum([e[0].numpy() for e in everyone], n * x.itemsize)
            res[name] = all(e[1].numpy().tobytes() == want.tobytes() for e in everyone)
    return {'cases': res, 'bit_exact': all(res.values()) if rank == 0 else None,
            'reference_order': lib.ddl_get_config(b'reference_order')}


_REAL_STDOUT = None


def emit(obj):
    """Write the ONE result line to the real stdout (libraries such as gloo print banners on
    fd 1; everything but this line goes to stderr)."""
    line = (json.dumps(obj) + '\n').encode()
    fd = _REAL_STDOUT if _REAL_STDOUT is not None else 1
    os.write(fd, line)


WATCHDOG_RC = 3           # a leg hung: the line (if any) carries `incomplete`
WATCHDOG_TEARDOWN_RC = 4  # the complete line was printed, then teardown hung


def _watchdog_selftest(args, state, rank, world):
    """CPU test hook for the N>1 watchdog (tests/test_bench_cpu.py): the ranks meet over gloo,
    rank 0 holds a stand-in headline (`selftest` marks it), then every rank but 0 stalls in leg
    'selftest_hang' while rank 0 waits for it in a barrier — a hung collective. The watchdog
    must end every rank with WATCHDOG_RC and rank 0's line must carry `incomplete`."""
    import torch.distributed as dist
    os.environ.setdefault('MASTER_ADDR', '127.0.0.1')
    os.environ.setdefault('MASTER_PORT', '29533')
    dist.init_process_group('gloo', rank=rank, world_size=world)
    state['out'] = {'metric': 'watchdog selftest', 'value': None, 'n_gpus': world, 'selftest': True}
    dist.barrier()
    state['leg'] = 'selftest_hang'
    if rank != 0:
        time.sleep(10 * args.watchdog_s + 60)
    dist.barrier()
    time.sleep(10 * args.watchdog_s + 60)
    os._exit(0)  # not reached while the watchdog works


def _free_port():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(('127.0.0.1', 0))
        return s.getsockname()[1]


def spawn_ranks(args):
    """`bench.py --gpus N` with no launcher: start N rank processes (RANK / LOCAL_RANK /
    WORLD_SIZE / MASTER_* set, as torch.distributed.run would) and exit with the first failing
    rank's code. The parent never imports torch or touches HIP (no GPU initialised here, so no
    exec hazards); rank 0's JSON line reaches this process's stdout directly."""
    import signal
    import subprocess
    port = _free_port()
    procs = []
    for r in range(args.gpus):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(args.gpus),
                   LOCAL_WORLD_SIZE=str(args.gpus), MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port),
                   DDL_BENCH_SPAWNED='1')
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env,
                                      start_new_session=True))
    deadline = time.time() + args.watchdog_s + 120
    rc = 0
    stop_at = None  # after a rank's watchdog fired, the others get a grace period to fire theirs
    try:
        live = list(procs)
        while live:
            for p in list(live):
                code = p.poll()
                if code is None:
                    continue
                live.remove(p)
                if code != 0 and rc == 0:
                    rc = code if code > 0 else 128 - code
                    grace = 15.0 if code in (WATCHDOG_RC, WATCHDOG_TEARDOWN_RC) else 0.0
                    sys.stderr.write(f'[bench] rank {procs.index(p)} exited with {code}; stopping the others'
                                     f'{f" in {grace:.0f} s" if grace else ""}\n')
                    stop_at = time.time() + grace
            if stop_at is not None and time.time() >= stop_at:
                for q in live:
                    os.killpg(q.pid, signal.SIGTERM)
                stop_at = float('inf')
            if time.time() > deadline:
                sys.stderr.write('[bench] ranks still running past the watchdog; killing them\n')
                for q in live:
                    os.killpg(q.pid, signal.SIGKILL)
                rc = rc or 124
                deadline = float('inf')
            time.sleep(0.05)
    finally:
        for q in procs:
            if q.poll() is None:
                os.killpg(q.pid, signal.SIGKILL)
                q.wait()
    return rc


def main():
    global _REAL_STDOUT
    args = parse()
    env_world = os.environ.get('WORLD_SIZE')
    if env_world is None and args.gpus > 1:
        sys.stdout.flush()
        sys.exit(spawn_ranks(args))
    sys.stdout.flush()
    _REAL_STDOUT = os.dup(1)
    os.dup2(2, 1)  # native and Python chatter -> stderr
    world = int(env_world) if env_world is not None else 1
    if world != args.gpus and not (args.force_multi and world == 1):
        sys.stderr.write(f'[bench] WORLD_SIZE={world} but --gpus {args.gpus}: refusing to print a line for a '
                         f'different world\n')
        sys.exit(2)
    if world <= 1 and not args.force_multi:
        single_gpu(args)
    else:
        multi_gpu(args)


if __name__ == '__main__':
    main()
