"""Process-group setup for the two parallel layouts the framework runs.

* **DP (agent replicas)** needs no collectives: one process per GPU, each a member of
  the input topic's consumer group (``runtime/pod.py`` picks the replica index; the
  topic runtimes assign partitions).  ``bench.py`` only uses the default group for its
  barrier / max-over-ranks timing.
* **TP (chat agent)**: ``torchrun --nproc-per-node tp`` inside one pod (rendered by
  ``core/k8s.py``).  Every rank joins one process group over RCCL (backend ``nccl`` on
  ROCm; point-to-point xGMI between the pod's GPUs); rank 0 runs the agent and the
  engine scheduler, the other ranks mirror its steps in the native executor's worker
  loop (``LLMEngine.worker_loop``).  Column/row-parallel weights and the all-reduces
  after o_proj / down_proj live in ``models/llama.py`` + ``ops/csrc/runner.hip``; the
  LM head stays vocab-parallel: each rank works on its own vocab slice and only per-row
  statistics, top-k/top-p histograms and candidates are all-reduced
  (``ops/csrc/sampling.hip`` tp_sample_*), never the [T, vocab] logits.

Reference: none -- the reference scales only by replica DP
(``DEPL/agents/AgentResourcesFactory.java:525-540``); TP is the MI355X addition for
Llama-3-70B (BASELINE config 5).
"""
from __future__ import annotations

import os
from typing import Optional

import torch
import torch.distributed as dist

from ..models.llama import TPInfo


def env_world() -> int:
    return int(os.environ.get("WORLD_SIZE", "1") or 1)


def env_rank() -> int:
    return int(os.environ.get("RANK", "0") or 0)


def local_device() -> str:
    """``cuda:$LOCAL_RANK`` when a GPU is present (one process per GPU), else ``cpu``."""
    if torch.cuda.is_available():
        return f"cuda:{int(os.environ.get('LOCAL_RANK', '0') or 0)}"
    return "cpu"


def init_tensor_parallel(world: Optional[int] = None, backend: Optional[str] = None) -> TPInfo:
    """Join (or reuse) the default process group and describe it as a TP group.

    ``MASTER_ADDR``/``MASTER_PORT``/``RANK``/``WORLD_SIZE`` come from torchrun.  The
    whole job is one TP group: a TP pod holds exactly ``tp`` ranks."""
    world = world or env_world()
    if world <= 1:
        return TPInfo()
    device = local_device()
    if not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if backend is None:
            backend = "nccl" if device.startswith("cuda") else "gloo"
        kw = {}
        if device.startswith("cuda"):
            torch.cuda.set_device(device)
            kw["device_id"] = torch.device(device)
        dist.init_process_group(backend, rank=env_rank(), world_size=world, **kw)
    if dist.get_world_size() != world:
        raise ValueError(f"tensor-parallel degree {world} != process-group size {dist.get_world_size()}")
    return TPInfo(dist.get_rank(), world, None)
