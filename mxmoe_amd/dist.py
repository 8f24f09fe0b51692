"""Multi-GPU partitioning of the GroupGEMM; one process per GPU, torch.distributed.

The reference has no multi-GPU path (no NCCL/MPI call site); this module adds two:

* expert-parallel weak scaling (``ep_shard``) — what bench.py measures at N > 1: the global batch is
  N x T tokens, routed experts are sharded by index over ranks (LPT on their FLOPs), each rank runs
  its experts with N x M_e rows plus the replicated shared expert on its local T tokens. No
  collective inside the GroupGEMM (dispatch/combine all-to-all belongs to the MoE layer).
* strong scaling of one call (``nslice_plan`` + ``allgather_outputs``): work items are
  (problem, N-slice) with slices a multiple of the tile width, assigned by LPT; the shared expert
  (50 % of the FLOPs of each call) is N-split so the speedup is not capped at 2x; per-rank C shards
  are exchanged with one all-gather of equal-size padded buffers over RCCL (xGMI).
"""
from __future__ import annotations

import dataclasses
from typing import Sequence

import torch

from .workload import QShape


def lpt_assign(costs: Sequence[float], world: int) -> list[int]:
    """Longest-processing-time: item -> rank, heaviest first onto the least-loaded rank."""
    load = [0.0] * world
    owner = [0] * len(costs)
    for i in sorted(range(len(costs)), key=lambda i: -costs[i]):
        r = min(range(world), key=lambda r: (load[r], r))
        owner[i] = r
        load[r] += costs[i]
    return owner


def ep_shard(layer: dict[str, list[QShape]], world: int, rank: int) -> dict[str, list[QShape]]:
    """Per-rank problem lists for expert-parallel weak scaling (last problem = shared expert)."""
    if world == 1:
        return layer
    routed = list(range(len(layer["gate_up"]) - 1))
    owner = lpt_assign([layer["gate_up"][e].flops + layer["down"][e].flops for e in routed], world)
    out = {}
    for gg in ("gate_up", "down"):
        lst = [QShape([s.M * world, s.N, s.K], s.w_bits, s.a_bits, s.gsize, s.sym)
               for e, s in ((e, layer[gg][e]) for e in routed) if owner[e] == rank]
        lst.append(layer[gg][-1])
        out[gg] = lst
    return out


@dataclasses.dataclass(frozen=True)
class NSlice:
    problem: int
    n0: int
    n1: int

    @property
    def width(self) -> int:
        return self.n1 - self.n0


def nslice_plan(shapes: Sequence[QShape], world: int, slice_n: int = 256, target_frac: float = 0.5) -> list[list[NSlice]]:
    """Split problems into N-slices (multiples of slice_n) so that no item exceeds target_frac of a
    rank's fair share, then LPT-assign them. Returns the work list per rank."""
    total = sum(s.flops for s in shapes)
    cap = max(1.0, target_frac * total / world)
    items: list[NSlice] = []
    for i, s in enumerate(shapes):
        if s.M == 0:
            continue
        parts = max(1, int(-(-s.flops // cap)))
        width = -(-s.N // parts)
        width = max(slice_n, -(-width // slice_n) * slice_n)
        for n0 in range(0, s.N, width):
            items.append(NSlice(i, n0, min(s.N, n0 + width)))
    cost = [2.0 * shapes[it.problem].M * it.width * shapes[it.problem].K for it in items]
    owner = lpt_assign(cost, world)
    return [[it for it, o in zip(items, owner) if o == r] for r in range(world)]


def shard_bytes(shapes: Sequence[QShape], work: Sequence[NSlice]) -> int:
    """fp16 output elements a rank produces for its work list."""
    return sum(shapes[w.problem].M * w.width for w in work)


def allgather_outputs(shapes: Sequence[QShape], plan: list[list[NSlice]], local: torch.Tensor,
                      outputs: Sequence[torch.Tensor], group=None) -> None:
    """All-gather every rank's packed C slices and scatter them into the full outputs.

    ``local`` holds this rank's slices packed back to back (work order, each [M, width] row-major);
    buffers are padded to the largest shard so one all_gather_into_tensor suffices (RCCL ring /
    xGMI; gloo on CPU in tests)."""
    import torch.distributed as dist

    world = len(plan)
    sizes = [shard_bytes(shapes, w) for w in plan]
    pad = max(sizes)
    buf = torch.zeros(pad, dtype=local.dtype, device=local.device)
    buf[: local.numel()] = local.reshape(-1)
    gathered = torch.empty(world * pad, dtype=local.dtype, device=local.device)
    dist.all_gather_into_tensor(gathered, buf, group=group)
    for r in range(world):
        off = r * pad
        for w in plan[r]:
            M = shapes[w.problem].M
            n = M * w.width
            outputs[w.problem][:M, w.n0:w.n1] = gathered[off:off + n].view(M, w.width)
            off += n
