"""ddl — MI355X-native gradient-bucket allreduce engine, PyTorch host side.

Mirror of the reference package `ddl` (LYL232/Experiment-Distributed-Deep-Learning,
src/py/ddl): `ddl.tensorflow.*` becomes `ddl.torch.*` with the same names — Communicator,
allreduce, allreduce_gradient and the data-parallel optimizer wrapper — backed by
lib/libddl_amd.so (HIP kernels for gfx950 + RCCL ring over xGMI) instead of the
TensorFlow-op + MPI library.
"""
