"""``torch.distributed``-style facade over this package's communicator.

    import ddp_practice_amd.distributed as dist
    dist.init_process_group("nccl", init_method="env://")   # RCCL underneath
    dist.reduce(t, 0, op=dist.ReduceOp.SUM)
    dist.destroy_process_group()

reference: /root/reference/ddp_main.py:69-73 (init_ddp), :108-109 (dist.reduce),
:170 (destroy_process_group).
"""
from __future__ import annotations

import torch
import torch.distributed as _tdist

from .parallel.comm import (barrier, default_comm, destroy_process_group, get_rank,  # noqa: F401
                            get_world_size, init_process_group, is_initialized, max_over_ranks)

ReduceOp = _tdist.ReduceOp


def all_reduce(tensor: torch.Tensor, op=ReduceOp.SUM, group=None, async_op: bool = False):
    (group or default_comm()).all_reduce_(tensor, op)
    return None


def reduce(tensor: torch.Tensor, dst: int, op=ReduceOp.SUM, group=None, async_op: bool = False):
    (group or default_comm()).reduce_(tensor, dst, op)
    return None


def broadcast(tensor: torch.Tensor, src: int, group=None, async_op: bool = False):
    (group or default_comm()).broadcast_(tensor, src)
    return None


def all_gather_into_tensor(output: torch.Tensor, input: torch.Tensor, group=None, async_op: bool = False):
    (group or default_comm()).all_gather_into_tensor(output, input)
    return None


def reduce_scatter_tensor(output: torch.Tensor, input: torch.Tensor, op=ReduceOp.SUM, group=None,
                          async_op: bool = False):
    (group or default_comm()).reduce_scatter_tensor(output, input, op)
    return None
