"""Data parallelism: communicator/process group, DDP (C++ reducer), SyncBatchNorm."""
from .comm import (Communicator, LocalCommunicator, RcclCommunicator, TorchCommunicator, XgmiCommunicator,  # noqa: F401,E501
                   default_comm, init_process_group)
from .ddp import DistributedDataParallel, compute_bucket_assignment  # noqa: F401
from .sync_bn import SyncBatchNorm, convert_sync_batchnorm  # noqa: F401
