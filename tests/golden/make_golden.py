#!/usr/bin/env python3
"""Generate the golden allreduce vectors under tests/golden/ (run in the build container).

The reference's data plane is a single MPI_Allreduce(MPI_SUM) call
(src/cpp/communicate/backend/mpi/MPICommunicator.cc:14-28). MPICH 3.3.2, the MPI the image
ships at /opt/conda, is run here through our own driver (oracle/mpi_allreduce_driver.c)
with `mpiexec -n P`, exactly as the reference calls it. The resulting fixture files are
data only: per case the P input buffers and MPICH's reduced output.

Cases:
  ref_test_P{2,4,8}       reference test/allreduce_test.py:13 — fp32[16] filled with rank;
                          known answer P(P-1)/2.
  survey_probe_P{2,8}     the survey's probe inputs through the reference path:
                          fp32 x_r[i] = 0.5(r+1) + (i mod 7), int32 r*1000 + (i mod 13).
  int32_rand_P{2,4,8}     full-range int32 (wrap-around), bit-exact at every P.
  fp32_randn_P{2,4,8}     N(0,1) fp32; bit-exact at P=2, error-bounded at P>2.
  fp32_exact_P8           k * 2^-10 with |k| < 2^12: exactly summable, bit-exact at P=8.
  fp64_randn_P{2,4}, int64_rand_P4, uint64_rand_P2.

  Full size (golden_fullsize.json, --fullsize): C3 fp32 P=8 and P=5 / P=7 at 64 Mi elements;
  hashes and samples only.

usage: python tests/golden/make_golden.py [--bigp | --fullsize]
       (--bigp: only golden_mpich_bigp.npz; --fullsize: only golden_fullsize.json)
"""
import json
import os
import subprocess
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
MPI_HOME = os.environ.get("MPI_HOME", "/opt/conda")
DRIVER = os.path.join(REPO, "oracle", "build", "mpi_allreduce_driver")

DT = {"float32": 1, "float64": 2, "int32": 3, "int64": 9, "uint64": 23}


def seed_for(rank):
    return 1234 + 7919 * rank


def make_inputs(kind, dtype, P, n):
    xs = []
    for r in range(P):
        rng = np.random.default_rng(seed_for(r))
        i = np.arange(n)
        if kind == "fill_rank":
            x = np.full(n, r, dtype=dtype)
        elif kind == "survey_probe":
            if dtype == "float32":
                x = (0.5 * (r + 1) + (i % 7)).astype(np.float32)
            else:
                x = (r * 1000 + (i % 13)).astype(np.int32)
        elif kind == "randint":
            info = np.iinfo(dtype)
            x = rng.integers(info.min, info.max, size=n, dtype=dtype, endpoint=True)
        elif kind == "randn":
            x = rng.standard_normal(n).astype(dtype)
        elif kind == "exact":
            k = rng.integers(-(2 ** 12) + 1, 2 ** 12, size=n)
            x = (k * 2.0 ** -10).astype(dtype)
        else:
            raise ValueError(kind)
        xs.append(np.ascontiguousarray(x, dtype=dtype))
    return np.stack(xs)


def run_mpich(inputs, dtype):
    P, n = inputs.shape
    with tempfile.TemporaryDirectory() as d:
        for r in range(P):
            inputs[r].tofile(os.path.join(d, f"in_{r}.bin"))
        env = dict(os.environ)
        env["LD_LIBRARY_PATH"] = os.path.join(MPI_HOME, "lib") + ":" + env.get("LD_LIBRARY_PATH", "")
        subprocess.run([os.path.join(MPI_HOME, "bin", "mpiexec"), "-n", str(P), DRIVER,
                        str(DT[dtype]), str(n), d], check=True, env=env, timeout=300)
        outs = [np.fromfile(os.path.join(d, f"out_{r}.bin"), dtype=dtype) for r in range(P)]
    for r in range(1, P):  # every rank must receive the same reduced buffer
        assert outs[r].tobytes() == outs[0].tobytes(), "MPICH ranks disagree"
    return outs[0]


CASES = [
    # name, kind, dtype, P, n
    ("ref_test_P2", "fill_rank", "float32", 2, 16),
    ("ref_test_P4", "fill_rank", "float32", 4, 16),
    ("ref_test_P8", "fill_rank", "float32", 8, 16),
    ("survey_probe_f32_P2", "survey_probe", "float32", 2, 1024),
    ("survey_probe_f32_P8", "survey_probe", "float32", 8, 1024),
    ("survey_probe_i32_P8", "survey_probe", "int32", 8, 1024),
    ("int32_rand_P2", "randint", "int32", 2, 1031),
    ("int32_rand_P4", "randint", "int32", 4, 1031),
    ("int32_rand_P8", "randint", "int32", 8, 1031),
    ("fp32_randn_P2", "randn", "float32", 2, 1031),
    ("fp32_randn_P4", "randn", "float32", 4, 1031),
    ("fp32_randn_P8", "randn", "float32", 8, 1031),
    ("fp32_exact_P8", "exact", "float32", 8, 1031),
    ("fp64_randn_P2", "randn", "float64", 2, 515),
    ("fp64_randn_P4", "randn", "float64", 4, 515),
    ("int64_rand_P4", "randint", "int64", 4, 515),
    ("uint64_rand_P2", "randint", "uint64", 2, 515),
    # non-power-of-two P on both sides of MPICH's 2048-byte algorithm switch (the order of the
    # additions differs there: binomial tree below, pre-fold + pairwise tree above)
    ("fp32_randn_P3_small", "randn", "float32", 3, 300),
    ("fp32_randn_P3", "randn", "float32", 3, 1031),
    ("fp32_randn_P5_small", "randn", "float32", 5, 512),
    ("fp32_randn_P5_switch", "randn", "float32", 5, 513),
    ("fp32_randn_P5", "randn", "float32", 5, 4099),
    ("fp32_randn_P6", "randn", "float32", 6, 4099),
    ("fp32_randn_P7_small", "randn", "float32", 7, 200),
    ("fp32_randn_P7", "randn", "float32", 7, 4099),
    ("fp64_randn_P5_small", "randn", "float64", 5, 256),
    ("fp64_randn_P5", "randn", "float64", 5, 257),
    ("fp64_randn_P8", "randn", "float64", 8, 515),
    ("fp32_randn_P8_large", "randn", "float32", 8, 16387),
]


# More ranks than one node's GPUs, one host: MPICH's orders beyond P = 8, the
# fold trees of more than 16 inputs, and MPICH's count < pof2 rule (recursive doubling above
# 2048 bytes when the element count is below the largest power of two <= P: P = 520, 257 fp64
# elements = 2056 bytes). Kept in their own file: the GPU runs P <= 64 virtual ranks.
BIGP_CASES = [
    ("fp32_randn_P17", "randn", "float32", 17, 3000),
    ("fp32_randn_P20_small", "randn", "float32", 20, 511),
    ("fp32_randn_P33", "randn", "float32", 33, 4099),
    ("fp64_randn_P33_small", "randn", "float64", 33, 255),
    ("int32_rand_P33", "randint", "int32", 33, 1031),
    ("fp64_randn_P520_count_lt_pof2", "randn", "float64", 520, 257),
]


def make_bigp():
    arrays, cases = {}, {}
    for name, kind, dtype, P, n in BIGP_CASES:
        x = make_inputs(kind, dtype, P, n)
        y = run_mpich(x, dtype)
        arrays[name + "__inputs"] = x
        arrays[name + "__output"] = y
        cases[name] = {"kind": kind, "dtype": dtype, "P": P, "n": n}
        print(f"{name}: P={P} n={n} {dtype} out[0]={y[0]}", flush=True)
    np.savez_compressed(os.path.join(HERE, "golden_mpich_bigp.npz"), **arrays)
    with open(os.path.join(HERE, "golden_manifest_bigp.json"), "w") as f:
        json.dump({"generator": "MPICH 3.3.2 MPI_Allreduce(MPI_SUM) via oracle/mpi_allreduce_driver.c, one host",
                   "seed": "numpy default_rng(1234 + 7919*rank)", "cases": cases}, f, indent=1, sort_keys=True)


# BASELINE.json configs[2] (C3) at its full size, and the non-power-of-two pre-fold at that size
# (VERDICT r5 next #1): 64 Mi fp32 elements (256 MiB) per rank. The 2-8 GiB of data are not
# committed: golden_fullsize.json keeps the generator, the seed rule, the sha256 of MPICH's
# output (identical on every rank) and sampled values; tests regenerate the inputs with
# fullsize_inputs() (numpy default_rng(seed_for(rank)).standard_normal, as "randn" above).
FULLSIZE_CASES = [
    ("c3_fp32_randn_P8_64Mi", "float32", 8, 64 << 20),
    ("fp32_randn_P5_64Mi", "float32", 5, 64 << 20),
    ("fp32_randn_P7_64Mi", "float32", 7, 64 << 20),
]
FULLSIZE_SAMPLE_IDX = [0, 1, 2, 1023, 1 << 20, (32 << 20) + 5, (64 << 20) - 2, (64 << 20) - 1]


def fullsize_inputs(P, n):
    """The full-size cases' rank inputs (same rule as make_inputs('randn', 'float32', P, n))."""
    return [np.random.default_rng(seed_for(r)).standard_normal(n).astype(np.float32) for r in range(P)]


def make_fullsize():
    import hashlib
    cases = {}
    for name, dtype, P, n in FULLSIZE_CASES:
        y = run_mpich(np.stack(fullsize_inputs(P, n)), dtype)
        cases[name] = {"dtype": dtype, "P": P, "n": n, "sha256": hashlib.sha256(y.tobytes()).hexdigest(),
                       "samples": {str(i): float(y[i]) for i in FULLSIZE_SAMPLE_IDX}}
        print(f"{name}: P={P} n={n} sha256={cases[name]['sha256'][:16]}", flush=True)
    with open(os.path.join(HERE, "golden_fullsize.json"), "w") as f:
        json.dump({"generator": "MPICH 3.3.2 MPI_Allreduce(MPI_SUM) via oracle/mpi_allreduce_driver.c, one host",
                   "reference_call": "src/cpp/communicate/backend/mpi/MPICommunicator.cc:14-28",
                   "seed": "numpy default_rng(1234 + 7919*rank).standard_normal(n).astype(float32)",
                   "output": "sha256 of MPICH's reduced buffer (every rank's output identical)",
                   "cases": cases}, f, indent=1, sort_keys=True)


def main():
    subprocess.run(["make", "-C", os.path.join(REPO, "oracle"), "mpi"], check=True)
    if "--fullsize" in sys.argv:
        make_fullsize()
        return 0
    make_bigp()
    if "--bigp" in sys.argv:
        return 0
    arrays, manifest = {}, {"generator": "MPICH 3.3.2 MPI_Allreduce(MPI_SUM) via oracle/mpi_allreduce_driver.c",
                            "reference_call": "src/cpp/communicate/backend/mpi/MPICommunicator.cc:14-28",
                            "seed": "numpy default_rng(1234 + 7919*rank)", "cases": {}}
    for name, kind, dtype, P, n in CASES:
        x = make_inputs(kind, dtype, P, n)
        y = run_mpich(x, dtype)
        arrays[name + "__inputs"] = x
        arrays[name + "__output"] = y
        manifest["cases"][name] = {"kind": kind, "dtype": dtype, "P": P, "n": n}
        print(f"{name}: P={P} n={n} {dtype} out[0]={y[0]}", flush=True)
    np.savez_compressed(os.path.join(HERE, "golden_mpich.npz"), **arrays)
    # Reference outputs recorded in SURVEY.md §4 (the survey ran the reference's own C++
    # path at P=2/8 on these inputs); kept as spot values, checked analytically in tests.
    manifest["survey_recorded"] = {
        "inputs": "fp32 x_r[i] = 0.5*(r+1) + (i mod 7); int32 x_r[i] = r*1000 + (i mod 13)",
        "P2": {"f32": {"0": 1.5, "1023": 3.5}},
        "P8": {"f32": {"0": 18.0, "1023": 26.0, "1048575": 42.0}, "i32": {"0": 28000}},
    }
    manifest["reference_test"] = {"file": "src/py/ddl/test/allreduce_test.py:5-17",
                                  "known_answer": "fp32[16] filled with rank -> P*(P-1)/2"}
    with open(os.path.join(HERE, "golden_manifest.json"), "w") as f:
        json.dump(manifest, f, indent=1, sort_keys=True)


if __name__ == "__main__":
    sys.exit(main())
