from ddl.torch.parallelism.data.callbacks import (  # noqa: F401
    InitialParametersBroadcast,
    LearningRateSchedule,
    LearningRateWarmup,
    MetricAverage,
)
from ddl.torch.parallelism.data.distributed_optimizer import (  # noqa: F401
    DataParallelismDistributedOptimizer,
    data_parallelism_distributed_optimizer_wrapper,
)
