"""Data parallelism over RCCL (xGMI) - see :mod:`gnnqc.parallel.dist`; opt-in one-shot peer
all-reduce over xGMI - :mod:`gnnqc.parallel.peer`."""
from .dist import (all_gather_var, all_reduce_, backend, barrier, broadcast_, broadcast_module, destroy,
                   init_distributed, is_initialized, is_main, max_over_ranks, rank, world_size)
from .peer import PeerAllReduce, make_peer_allreduce, peer_enabled

__all__ = ["init_distributed", "destroy", "barrier", "all_reduce_", "broadcast_", "broadcast_module",
           "all_gather_var", "max_over_ranks", "world_size", "rank", "is_main", "is_initialized", "backend",
           "PeerAllReduce", "make_peer_allreduce", "peer_enabled"]
