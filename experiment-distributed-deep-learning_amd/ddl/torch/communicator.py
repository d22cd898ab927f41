"""Communicator handle (mirror of reference src/py/ddl/tensorflow/communicator.py:4-59).

The reference initialises MPI when its library is loaded (MPIBackend.cc:77-97, launched by
`mpirun`). Here one process drives one GPU and the launcher is `torch.distributed.run`
(RANK / WORLD_SIZE / LOCAL_RANK / MASTER_ADDR / MASTER_PORT): `init()` — called lazily by
`Communicator.world()` — creates the RCCL bootstrap id on rank 0, distributes it and every
rank's control-channel endpoint through a gloo process group, then builds the world
communicator and its token ring.
"""
import ctypes
import os

import torch

from ddl.torch.cpp_backend import CPPBackend, check


def _env_int(name: str, default: int) -> int:
    v = os.environ.get(name)
    return int(v) if v not in (None, '') else default


def init(rank: int = None, size: int = None, device: int = None) -> None:
    """Create the world communicator for this process (idempotent)."""
    api = CPPBackend.c_api()
    if api.ddl_is_initialized():
        return
    rank = _env_int('RANK', 0) if rank is None else rank
    size = _env_int('WORLD_SIZE', 1) if size is None else size
    device = _env_int('LOCAL_RANK', 0) if device is None else device
    torch.cuda.set_device(device)
    if size == 1:
        check(api.ddl_init_single(device), 'ddl_init_single')
        return
    import torch.distributed as dist
    if not dist.is_initialized():
        os.environ.setdefault('MASTER_ADDR', '127.0.0.1')
        dist.init_process_group('gloo', rank=rank, world_size=size)
    uid = ctypes.create_string_buffer(128)
    if rank == 0:
        check(api.ddl_get_unique_id(uid, 128), 'ddl_get_unique_id')
    box = [uid.raw if rank == 0 else None]
    dist.broadcast_object_list(box, src=0)
    uid = ctypes.create_string_buffer(box[0], 128)
    check(api.ddl_init(rank, size, device, uid, 128), 'ddl_init')
    ep = ctypes.create_string_buffer(256)
    check(api.ddl_control_listen(ep, 256), 'ddl_control_listen')
    eps = [None] * size
    dist.all_gather_object(eps, ep.value.decode())
    check(api.ddl_control_connect(';'.join(eps).encode()), 'ddl_control_connect')


def finalize() -> None:
    check(CPPBackend.c_api().ddl_finalize(), 'ddl_finalize')
    Communicator._Communicator__world = None


class Communicator:
    """A communication domain; `id` is the engine's 64-bit handle (reference: MPI_Comm*)."""
    __world = None

    def __init__(self, communicator_id: int):
        self.__id = communicator_id
        self.__rank = None
        self.__size = None

    @property
    def id(self):
        return self.__id

    @property
    def rank(self) -> int:
        if self.__rank is None:
            self.__rank = CPPBackend.c_api().communicator_rank(self.id)
            if self.__rank < 0:
                check(2, 'communicator_rank')
        return self.__rank

    @property
    def size(self) -> int:
        if self.__size is None:
            self.__size = CPPBackend.c_api().communicator_size(self.id)
            if self.__size < 0:
                check(2, 'communicator_size')
        return self.__size

    def split_communicator(self, color: int, key: int = None) -> 'Communicator':
        """Collective split by color; `key` orders ranks (default: rank in this domain)."""
        if key is None:
            key = self.rank
        new_id = CPPBackend.c_api().split_communicator(self.id, color, key)
        if new_id == 0:
            check(2, 'split_communicator')
        return Communicator(new_id)

    def detach(self) -> None:
        CPPBackend.c_api().detach_communicator(self.id)

    @classmethod
    def world(cls) -> 'Communicator':
        if cls.__world is None:
            init()
            cid = CPPBackend.c_api().world_communicator()
            if cid == 0:
                check(6, 'world_communicator')
            cls.__world = cls(cid)
        return cls.__world
