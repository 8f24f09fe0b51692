"""Multi-GPU partitioning of the GroupGEMM; one process per GPU, torch.distributed.

The reference has no multi-GPU path (no NCCL/MPI call site); this module adds three:

* expert-parallel strong scaling of one layer (``ep_layer_plan`` + ``EPLayerStep``) — bench.py's
  N > 1 headline, north_star's "experts shard by index across the GPUs with an RCCL all-gather of
  per-shard outputs": routed experts are sharded by index (LPT on their gate_up + down FLOPs), the
  shared expert by token rows (sized so every rank's FLOPs even out); each rank runs gate_up and
  down for its share — the gate_up output is the down call's input in the layer and stays on its
  rank — and the layer's outputs (down C, packed into one shard per rank) are exchanged with one
  all_gather_into_tensor over RCCL / xGMI.
* strong scaling by N-slices (``nslice_plan`` + ``ShardedCall`` + ``ShardedLayerStep``) — an extra:
  work items are (problem, N-slice) of each call; every call's C (gate_up included) is all-gathered,
  the gate_up gather on a second stream while the down call computes.
* expert-parallel weak scaling (``ep_shard``) — an extra: the global batch is N x T tokens, routed
  experts are sharded by index, each rank runs its experts with N x M_e rows plus the replicated
  shared expert on its local T tokens; no collective (dispatch / combine belongs to the MoE layer).
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


@dataclasses.dataclass(frozen=True)
class RowItem:
    """Rows [m0, m1) of one problem (a whole routed expert, or a row slice of the shared expert)."""

    problem: int
    m0: int
    m1: int

    @property
    def rows(self) -> int:
        return self.m1 - self.m0


def ep_layer_plan(gate_up: Sequence[QShape], down: Sequence[QShape], world: int, shared: bool = True,
                  row_align: int = 64) -> list[list[RowItem]]:
    """Per-rank work of one layer split by expert (the same items for the gate_up and down calls).

    Routed experts (every problem but the last when ``shared``) go whole to ranks by LPT on their
    gate_up + down FLOPs; the shared expert's token rows are cut into one contiguous slice per rank
    (multiples of ``row_align`` rows, the last slice takes the rest) sized to fill each rank up to
    an even share of the layer's FLOPs."""
    P = len(gate_up)
    nr = P - 1 if shared else P
    routed = [i for i in range(nr) if gate_up[i].M > 0]
    cost = [float(gate_up[i].flops + down[i].flops) for i in routed]
    owner = lpt_assign(cost, world)
    load = [0.0] * world
    work: list[list[RowItem]] = [[] for _ in range(world)]
    for i, o, c in zip(routed, owner, cost):
        work[o].append(RowItem(i, 0, gate_up[i].M))
        load[o] += c
    if shared and P and gate_up[-1].M > 0:
        M = gate_up[-1].M
        per_row = float(gate_up[-1].flops + down[-1].flops) / M
        target = (sum(load) + per_row * M) / world
        want = [max(0.0, (target - ld) / per_row) for ld in load]
        tot = sum(want)
        want = [w * M / tot for w in want] if tot > 0 else [M / world] * world
        bounds, acc = [0], 0.0
        for r in range(world):
            acc += want[r]
            b = M if r == world - 1 else min(M, int(round(acc / row_align)) * row_align)
            bounds.append(max(b, bounds[-1]))
        for r in range(world):
            if bounds[r + 1] > bounds[r]:
                work[r].append(RowItem(P - 1, bounds[r], bounds[r + 1]))
    return work


def ep_shard_elems(shapes: Sequence[QShape], work: Sequence[RowItem]) -> int:
    """fp16 output elements of one call that a rank's row items produce."""
    return sum(w.rows * shapes[w.problem].N for w in work)


def ep_scatter(shapes: Sequence[QShape], plan: list[list[RowItem]], gathered: torch.Tensor, pad: int,
               outputs: Sequence[torch.Tensor]) -> None:
    """Place an all-gathered buffer (rank r's packed shard at r * pad, items in work order, each a
    [rows, N] row-major block) into the full per-problem outputs."""
    for r, items in enumerate(plan):
        off = r * pad
        for w in items:
            n = w.rows * shapes[w.problem].N
            outputs[w.problem][w.m0:w.m1] = gathered[off:off + n].view(w.rows, shapes[w.problem].N)
            off += n


def ep_layer_chunks(plan: list[list[RowItem]], gate_up: Sequence[QShape], down: Sequence[QShape], chunks: int,
                    row_align: int = 64) -> list[list[list[RowItem]]]:
    """Cut every rank's work into `chunks` groups of about equal FLOPs (a shared-expert row slice is
    cut into `chunks` row parts first, in multiples of `row_align`; then LPT): returns one per-rank
    plan per chunk, so that chunk c's outputs can be all-gathered while chunk c + 1 computes."""
    if chunks <= 1:
        return [plan]
    out: list[list[list[RowItem]]] = [[[] for _ in plan] for _ in range(chunks)]
    for r, items in enumerate(plan):
        pieces = []
        for w in items:
            if w.rows >= chunks * row_align and w.problem == len(gate_up) - 1:
                step = -(-w.rows // chunks // row_align) * row_align
                pieces += [RowItem(w.problem, m, min(w.m1, m + step)) for m in range(w.m0, w.m1, step)]
            else:
                pieces.append(w)
        cost = [float(w.rows) * (gate_up[w.problem].N * gate_up[w.problem].K + down[w.problem].N * down[w.problem].K)
                for w in pieces]
        for w, c in zip(pieces, lpt_assign(cost, chunks)):
            out[c][r].append(w)
    return out


XGMI_LINK_GBS = 64.0  # effective all-gather GB/s per xGMI link and direction (of ~153 GB/s raw per link)
CHUNK_OVERHEAD_MS = 0.015  # per extra chunk: two more launches + one more ragged finish per call


def gather_ms_model(bytes_received: float, world: int) -> float:
    """Modelled all-gather time: on a fully connected node every rank receives each peer's shard over
    its own xGMI link, so (world - 1) links carry the bytes in parallel."""
    if world <= 1:
        return 0.0
    return bytes_received / ((world - 1) * XGMI_LINK_GBS * 1e9) * 1e3


def choose_chunks(t_compute_ms: float, t_gather_ms: float, max_chunks: int = 8,
                  overhead_ms: float = CHUNK_OVERHEAD_MS) -> int:
    """Chunk count of EPLayerStep's compute / all-gather pipeline. With c chunks, chunk i's gather
    runs beside chunk i+1's compute, so the step takes about
        max(Tc, Tg) + min(Tc, Tg) / c + (c - 1) * overhead
    (the longer stream, plus the first compute or last gather chunk that nothing hides, plus the
    cost of cutting the calls finer); returns the c in [1, max_chunks] that minimises it."""
    lo, hi = sorted((max(t_compute_ms, 0.0), max(t_gather_ms, 0.0)))
    best, best_t = 1, None
    for c in range(1, max_chunks + 1):
        t = hi + lo / c + (c - 1) * overhead_ms
        if best_t is None or t < best_t - 1e-12:
            best, best_t = c, t
    return best


class EPLayerStep:
    """This rank's part of one layer split by ``ep_layer_plan``: per chunk (``ep_layer_chunks``) one
    planned gate_up call and one down call over its row items, and one all_gather_into_tensor of
    the chunk's packed down outputs. With chunks > 1 the gather of chunk c runs on a second stream
    while chunk c + 1 computes (RCCL runs the gathers in issue order on that stream).

    gate_up C is written into the full-size C tensors (rows of this rank's items only: it feeds the
    down call of the same rank in the layer); down C goes into a packed local shard so the exchange
    moves one contiguous buffer per rank and chunk."""

    def __init__(self, gate_up, down, world: int, rank: int, variant: Optional[int] = None, group=None,
                 shared: bool = True, chunks: int = 1):
        from .groupgemm import GroupGemm
        from .harness import slice_rows

        self.shapes_gu, self.shapes_dn = list(gate_up.shapes), list(down.shapes)
        self.world, self.rank, self.group = world, rank, group
        self.plan = ep_layer_plan(self.shapes_gu, self.shapes_dn, world, shared)
        self.chunk_plans = ep_layer_chunks(self.plan, self.shapes_gu, self.shapes_dn, chunks)
        dev = down.problems[0].C.device
        self.parts = []  # per chunk: (gate_up call, down call, local shard, gathered, pad)
        for cplan in self.chunk_plans:
            pad = max(max(ep_shard_elems(self.shapes_dn, w) for w in cplan), 1)
            local = torch.zeros(pad, dtype=torch.float16, device=dev)
            gathered = torch.empty(world * pad, dtype=torch.float16, device=dev)
            mine = cplan[rank]
            gu = [slice_rows(gate_up.problems[w.problem], w.m0, w.m1) for w in mine]
            dn, off = [], 0
            for w in mine:
                p = down.problems[w.problem]
                n = w.rows * p.N
                dn.append(slice_rows(p, w.m0, w.m1, C=local[off:off + n].view(w.rows, p.N)))
                off += n
            self.parts.append((GroupGemm(gu, variant=variant, device=dev) if gu else None,
                               GroupGemm(dn, variant=variant, device=dev) if dn else None, local, gathered, pad))
        self.pad = sum(p[4] for p in self.parts)
        mine = self.plan[rank]
        self.flops_local = {"gate_up": sum(2 * w.rows * self.shapes_gu[w.problem].N * self.shapes_gu[w.problem].K
                                           for w in mine),
                            "down": sum(2 * w.rows * self.shapes_dn[w.problem].N * self.shapes_dn[w.problem].K
                                        for w in mine)}
        self.comm = torch.cuda.Stream(device=dev) if dev.type == "cuda" and len(self.parts) > 1 else None
        self.evs = [torch.cuda.Event() for _ in self.parts] if self.comm is not None else []

    @property
    def gu(self):
        return self.parts[0][0]

    @property
    def dn(self):
        return self.parts[0][1]

    def compute(self, stream: Optional[torch.cuda.Stream] = None) -> None:
        for gu, dn, *_ in self.parts:
            for gg in (gu, dn):
                if gg is not None:
                    gg.launch(stream)

    def gather(self) -> None:
        for *_, local, gathered, _pad in self.parts:
            _all_gather(gathered, local, self.group)

    def __call__(self, stream: torch.cuda.Stream) -> None:
        if self.comm is None:
            self.compute(stream)
            with torch.cuda.stream(stream):
                self.gather()
            return
        for (gu, dn, local, gathered, _pad), ev in zip(self.parts, self.evs):
            for gg in (gu, dn):
                if gg is not None:
                    gg.launch(stream)
            ev.record(stream)
            self.comm.wait_event(ev)
            with torch.cuda.stream(self.comm):
                _all_gather(gathered, local, self.group)
        stream.wait_stream(self.comm)

    def scatter(self, outputs: Sequence[torch.Tensor]) -> None:
        for cplan, (*_, gathered, pad) in zip(self.chunk_plans, self.parts):
            ep_scatter(self.shapes_dn, cplan, gathered, pad, outputs)
