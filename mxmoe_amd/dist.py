"""Multi-GPU partitioning of the GroupGEMM; one process per GPU, torch.distributed.

The reference has no multi-GPU path (no NCCL/MPI call site); this module adds two:

* expert-parallel weak scaling (``ep_shard``) — what bench.py measures at N > 1: the global batch is
  N x T tokens, routed experts are sharded by index over ranks (LPT on their FLOPs), each rank runs
  its experts with N x M_e rows plus the replicated shared expert on its local T tokens. No
  collective inside the GroupGEMM (dispatch/combine all-to-all belongs to the MoE layer).
* strong scaling of one layer (``nslice_plan`` + ``ShardedCall`` + ``ShardedLayerStep``) — what
  bench.py measures at N > 1: work items are (problem, N-slice) with slices a multiple of the tile
  width, assigned by LPT; the shared expert (50 % of the FLOPs of each call) is N-split so the
  speedup is not capped at 2x; every rank writes its C slices packed into one padded local shard and
  the shards are exchanged with one all_gather_into_tensor per call over RCCL (xGMI). The gate_up
  gather runs on a second stream while the down call computes.
"""
from __future__ import annotations

import dataclasses
from typing import Optional, Sequence

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


def _all_gather(out: torch.Tensor, inp: torch.Tensor, group=None) -> None:
    """all_gather_into_tensor on the device the tensors live on; with a gloo group and CUDA tensors
    (the multi-rank rehearsal on one GPU) it is staged through host memory."""
    import torch.distributed as dist

    if inp.is_cuda and dist.get_backend(group) == "gloo":
        host = torch.empty(out.numel(), dtype=out.dtype)
        dist.all_gather_into_tensor(host, inp.cpu(), group=group)
        out.copy_(host)
    else:
        dist.all_gather_into_tensor(out, inp, group=group)


class ShardedCall:
    """This rank's part of one GroupGEMM call split by ``nslice_plan``.

    Each work item (problem, [n0, n1)) runs as an N' = n1 - n0 problem whose C is a [M, N'] block of
    one packed local shard (work order, row-major blocks) — the all-gather then moves one contiguous
    buffer per rank, no repacking on the GPU. ``scatter`` places a gathered buffer into full C
    tensors (verification only; the layer's consumer can read the packed shards directly)."""

    def __init__(self, inputs, world: int, rank: int, variant: Optional[int] = None, group=None):
        from .groupgemm import GroupGemm
        from .harness import slice_scale_b

        self.shapes = list(inputs.shapes)
        self.world, self.rank, self.group = world, rank, group
        self.plan = nslice_plan(self.shapes, world)
        self.sizes = [shard_bytes(self.shapes, w) for w in self.plan]
        self.pad = max(self.sizes) if self.sizes else 0
        dev = inputs.problems[0].C.device
        self.local = torch.zeros(max(self.pad, 1), dtype=torch.float16, device=dev)
        self.gathered = torch.empty(world * max(self.pad, 1), dtype=torch.float16, device=dev)
        mine, off = [], 0
        for w in self.plan[rank]:
            p = inputs.problems[w.problem]
            n = p.M * w.width
            mine.append(dataclasses.replace(p, B=p.B[w.n0:w.n1], N=w.width, ldc=0,
                                            C=self.local[off:off + n].view(max(p.M, 1), w.width)
                                            if p.M else self.local[:w.width].view(1, w.width),
                                            scale_b=slice_scale_b(p, w.n0, w.n1)))
            off += n
        self.part = GroupGemm(mine, variant=variant, device=dev) if mine else None
        self.flops_local = sum(2 * self.shapes[w.problem].M * w.width * self.shapes[w.problem].K for w in self.plan[rank])

    def compute(self, stream: Optional[torch.cuda.Stream] = None) -> None:
        if self.part is not None:
            self.part.launch(stream)

    def gather(self) -> None:
        """All-gather the padded shards (on the current stream)."""
        _all_gather(self.gathered, self.local, self.group)

    def scatter(self, outputs: Sequence[torch.Tensor]) -> None:
        for r in range(self.world):
            off = r * self.pad
            for w in self.plan[r]:
                M = self.shapes[w.problem].M
                n = M * w.width
                if M:
                    outputs[w.problem][:M, w.n0:w.n1] = self.gathered[off:off + n].view(M, w.width)
                off += n


class ShardedLayerStep:
    """One layer step on N ranks: gate_up part, its all-gather on a comm stream overlapped with the
    down part (SURVEY.md §8(e) "gather gate_up shards while down runs"), then the down all-gather.
    RCCL runs collectives of one communicator in issue order, so the down gather follows the gate_up
    gather; the main stream waits for both before the step ends."""

    def __init__(self, gate_up: ShardedCall, down: ShardedCall, overlap: bool = True):
        self.gu, self.dn = gate_up, down
        self.overlap = overlap
        self.comm = torch.cuda.Stream(device=gate_up.local.device) if gate_up.local.is_cuda else None
        self.ev = torch.cuda.Event() if self.comm is not None else None

    def compute_only(self, stream: torch.cuda.Stream) -> None:
        self.gu.compute(stream)
        self.dn.compute(stream)

    def __call__(self, stream: torch.cuda.Stream) -> None:
        self.gu.compute(stream)
        if self.overlap and self.comm is not None:
            self.ev.record(stream)
            self.comm.wait_event(self.ev)
            with torch.cuda.stream(self.comm):
                self.gu.gather()
            self.dn.compute(stream)
            with torch.cuda.stream(stream):
                self.dn.gather()
            stream.wait_stream(self.comm)
        else:
            with torch.cuda.stream(stream):
                self.gu.gather()
            self.dn.compute(stream)
            with torch.cuda.stream(stream):
                self.dn.gather()
