from ddl.torch.parallelism.data.callbacks import InitialParametersBroadcast, MetricAverage  # noqa: F401
from ddl.torch.parallelism.data.distributed_optimizer import (  # noqa: F401
    DataParallelismDistributedOptimizer,
    data_parallelism_distributed_optimizer_wrapper,
)
