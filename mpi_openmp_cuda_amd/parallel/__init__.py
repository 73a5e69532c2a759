"""Distributed layer: partitioning, torch.distributed (RCCL/gloo) pipeline, node-shared windows."""
