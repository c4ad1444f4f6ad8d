"""Date-sharded data parallelism over RCCL (torch.distributed, backend "nccl") or gloo (CPU)."""
