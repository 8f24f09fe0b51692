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


def gather_ms_model(bytes_received: float, world: int, link_gbs: float = XGMI_LINK_GBS) -> float:
    """Modelled all-gather time: on a fully connected node every rank receives each peer's shard over
    its own xGMI link, so (world - 1) links carry the bytes in parallel (link_gbs: effective GB/s per
    link and direction — an assumption, never measured here: no 8-GPU run has happened)."""
    if world <= 1:
        return 0.0
    return bytes_received / ((world - 1) * link_gbs * 1e9) * 1e3


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


# ------------------------------------------------------------------ combine before the exchange
#
# EPLayerStep all-gathers every rank's per-expert down C (the layer's 168 MB of expert outputs at
# qwen2_moe bs 8192: each rank receives ~152 MB at N = 8). What the MoE layer's consumer needs is the
# top-k weighted combine of those rows, [T, hidden] fp16 (33.5 MB). The token-owner exchange below
# sends each routed output row only to the rank that owns its token (an all-to-all of ~1/N of the
# rows), combines there in top-k order with the shared expert's rows that rank computed itself
# (mxmoe_moe_combine: the oracle's fma order, so the result is bit-identical to one-GPU
# MoEFFN.forward), and optionally all-gathers the combined [T, hidden] output.


@dataclasses.dataclass
class TokenRouting:
    """Host routing of one layer: topk_ids int32 [T, topk] (-1 = a dropped choice: the workload rule
    int(p * T * topk) leaves sum(M_e) a few slots short of T * topk) and weights float32 [T, topk]
    (0 for a dropped choice)."""

    topk_ids: "np.ndarray"
    weights: "np.ndarray"
    E: int

    @property
    def T(self) -> int:
        return int(self.topk_ids.shape[0])

    @property
    def topk(self) -> int:
        return int(self.topk_ids.shape[1])

    def slots(self):
        """The slot order of mxmoe_moe_route (stable sort by expert; dropped choices last):
        (sorted_expert, perm_token, inv_slot, counts[E], first_slot[E])."""
        import numpy as np

        flat = self.topk_ids.reshape(-1).astype(np.int64)
        key = np.where(flat < 0, self.E, flat)
        order = np.argsort(key, kind="stable")
        inv = np.empty_like(order)
        inv[order] = np.arange(order.size)
        counts = np.bincount(key, minlength=self.E + 1)[: self.E]
        first = np.concatenate([[0], np.cumsum(counts)[:-1]]).astype(np.int64)
        return key[order], order // self.topk, inv, counts, first


def synthetic_routing(counts: Sequence[int], T: int, topk: int, seed: int = 0) -> TokenRouting:
    """A routing of T tokens whose per-expert row counts are exactly ``counts`` (the workload's M_e):
    expert e's id appears M_e times, the T * topk - sum(M_e) other choices are dropped (-1), all in a
    seeded random order; weights are seeded positive f32 values normalised per token (0 if dropped)."""
    import numpy as np

    n = T * topk
    ids = np.concatenate([np.full(int(c), e, dtype=np.int32) for e, c in enumerate(counts)] +
                         [np.full(n - int(sum(counts)), -1, dtype=np.int32)])
    if ids.size != n:
        raise ValueError(f"sum of counts {sum(counts)} exceeds T * topk = {n}")
    rng = np.random.default_rng(seed)
    ids = ids[rng.permutation(n)].reshape(T, topk)
    w = rng.random((T, topk), dtype=np.float32) + np.float32(0.05)
    w = np.where(ids < 0, np.float32(0), w)
    s = w.sum(axis=1, keepdims=True)
    w = (w / np.where(s > 0, s, 1)).astype(np.float32)
    return TokenRouting(ids, w, len(counts))


@dataclasses.dataclass
class CombinePlan:
    """Who sends which down-output rows to whom (identical on every rank; numpy, host)."""

    world: int
    topk: int
    token_range: list          # per rank (t0, t1): the tokens it owns (= its shared-expert rows)
    shared_base: list          # per rank: first row of its shared-expert rows in its packed down shard (-1: none)
    send_rows: list            # send_rows[s][d]: rank s's packed-shard rows for rank d, in send order
    inv_local: list            # per rank d: int32 [n_d * topk] rows of d's receive buffer (R_d = a zero row)
    weights_local: list        # per rank d: float32 [n_d, topk]
    recv_rows: list            # per rank d: R_d rows received in all

    def split_sizes(self, rank: int):
        """(rows rank sends to each rank, rows it receives from each rank)."""
        return ([len(self.send_rows[rank][d]) for d in range(self.world)],
                [len(self.send_rows[s][rank]) for s in range(self.world)])

    def bytes_received(self, H: int) -> dict:
        """Per-rank bytes received (fp16 rows of H) by the all-to-all (rows from other ranks) and by
        the all-gather of the combined output ([T, H] minus the rank's own tokens)."""
        T = self.token_range[-1][1] if self.token_range else 0
        a2a = [2 * H * sum(len(self.send_rows[s][d]) for s in range(self.world) if s != d) for d in range(self.world)]
        pad = max((t1 - t0 for t0, t1 in self.token_range), default=0)
        ag = [2 * H * (self.world - 1) * pad for _ in range(self.world)]
        return {"all_to_all": a2a, "allgather_out": ag, "T": T}


def ep_combine_plan(plan: list[list[RowItem]], down: Sequence[QShape], routing: TokenRouting,
                    shared: bool = True) -> CombinePlan:
    """The token-owner exchange of an ep_layer_plan: rank d owns the tokens of its shared-expert row
    slice (or an even token split without a shared expert); every routed down-output row goes to the
    owner of its token; the owner's receive buffer holds rows source by source, each source's rows in
    its send order (work order, then row order), plus one zero row for dropped choices."""
    import numpy as np

    world = len(plan)
    P = len(down)
    E = P - 1 if shared else P
    T, topk = routing.T, routing.topk
    if routing.E != E:
        raise ValueError(f"routing has {routing.E} experts, the layer {E}")
    sorted_e, perm_token, inv, counts, first = routing.slots()
    for e in range(E):
        if int(counts[e]) != down[e].M:
            raise ValueError(f"expert {e}: routing has {int(counts[e])} rows, the layer {down[e].M}")
    if shared and down[-1].M != T:
        raise ValueError("the shared expert's rows must be the T tokens")
    # token ranges: the shared-expert slices (contiguous, in rank order), else an even split
    rng_ = [(0, 0)] * world
    base_sh = [-1] * world
    if shared:
        for r, items in enumerate(plan):
            base = 0
            for w in items:
                if w.problem == P - 1:
                    rng_[r] = (w.m0, w.m1)
                    base_sh[r] = base
                base += w.rows
        lo = 0
        for r in range(world):  # ranks without shared rows own an empty range at the boundary
            if rng_[r][1] == rng_[r][0]:
                rng_[r] = (lo, lo)
            lo = rng_[r][1]
    else:
        rng_ = [(T * r // world, T * (r + 1) // world) for r in range(world)]
    if rng_[0][0] != 0 or rng_[-1][1] != T or any(rng_[r][1] != rng_[r + 1][0] for r in range(world - 1)):
        raise ValueError(f"token ranges {rng_} do not tile [0, {T})")
    owner = np.empty(T, dtype=np.int64)
    for r, (t0, t1) in enumerate(rng_):
        owner[t0:t1] = r
    # send lists and where each routed slot lands in its owner's receive buffer
    send = [[None] * world for _ in range(world)]
    slot_src = np.full(int(counts.sum()), -1, dtype=np.int64)
    slot_idx = np.full(int(counts.sum()), -1, dtype=np.int64)
    for s, items in enumerate(plan):
        rows_s, slots_s = [], []
        base = 0
        for w in items:
            if w.problem < E:
                sl = first[w.problem] + np.arange(w.m0, w.m1)
                rows_s.append(base + np.arange(w.rows))
                slots_s.append(sl)
            base += w.rows
        rows_s = np.concatenate(rows_s) if rows_s else np.zeros(0, np.int64)
        slots_s = np.concatenate(slots_s) if slots_s else np.zeros(0, np.int64)
        dest = owner[perm_token[slots_s]] if slots_s.size else np.zeros(0, np.int64)
        for d in range(world):
            m = dest == d
            send[s][d] = rows_s[m]
            slot_src[slots_s[m]] = s
            slot_idx[slots_s[m]] = np.arange(int(m.sum()))
    inv_local, w_local, recv_rows = [], [], []
    for d in range(world):
        off = np.cumsum([0] + [len(send[s][d]) for s in range(world)])
        R = int(off[-1])
        t0, t1 = rng_[d]
        sl = inv.reshape(T, topk)[t0:t1].reshape(-1)
        routed = sl < slot_src.size
        pos = np.full(sl.size, R, dtype=np.int64)  # dropped choices read the zero row
        pos[routed] = off[slot_src[sl[routed]]] + slot_idx[sl[routed]]
        inv_local.append(pos.astype(np.int32))
        w_local.append(np.ascontiguousarray(routing.weights[t0:t1], dtype=np.float32))
        recv_rows.append(R)
    return CombinePlan(world, topk, rng_, base_sh, send, inv_local, w_local, recv_rows)


def _all_to_all_rows(recv: torch.Tensor, send: torch.Tensor, out_splits, in_splits, group=None) -> None:
    """all_to_all_single over rows (RCCL on the node; staged through host memory under gloo with CUDA
    tensors, the one-GPU rehearsal)."""
    import torch.distributed as dist

    if send.is_cuda and dist.get_backend(group) == "gloo":
        host = torch.empty(recv.shape, dtype=recv.dtype)
        dist.all_to_all_single(host, send.cpu(), out_splits, in_splits, group=group)
        recv.copy_(host)
    else:
        dist.all_to_all_single(recv, send, out_splits, in_splits, group=group)


class CombineExchange:
    """This rank's side of the token-owner exchange (ep_combine_plan): gather the rows to send from
    the packed down shard (one index_select), exchange them with one all_to_all_single, combine the
    owned tokens (``combine_fn``, default the HIP mxmoe_moe_combine), and — with ``gather_output`` —
    all-gather the combined [T, H] output so every rank holds it (padded to the largest token range)."""

    def __init__(self, cplan: CombinePlan, rank: int, H: int, device, combine_fn=None, gather_output: bool = True,
                 group=None):
        self.cp, self.rank, self.H, self.group = cplan, rank, H, group
        self.gather_output = gather_output
        dev = torch.device(device)
        import numpy as np

        self.send_idx = torch.from_numpy(
            np.concatenate([cplan.send_rows[rank][d] for d in range(cplan.world)]).astype(np.int64)).to(dev)
        self.in_splits, self.out_splits = cplan.split_sizes(rank)
        R = cplan.recv_rows[rank]
        self.send = torch.empty(int(self.send_idx.numel()), H, dtype=torch.float16, device=dev)
        self.recv = torch.zeros(R + 1, H, dtype=torch.float16, device=dev)  # last row: zero (dropped choices)
        self.inv = torch.from_numpy(cplan.inv_local[rank]).to(dev)
        self.w = torch.from_numpy(cplan.weights_local[rank]).to(dev)
        t0, t1 = cplan.token_range[rank]
        self.n = t1 - t0
        self.pad = max(t1 - t0 for t0, t1 in cplan.token_range)
        self.out = torch.empty(max(self.pad, 1), H, dtype=torch.float16, device=dev)
        self.gathered = torch.empty(cplan.world * max(self.pad, 1), H, dtype=torch.float16, device=dev)
        if combine_fn is None:
            from .moe import combine_into

            def combine_fn(out, y, inv, w, shared, topk):
                combine_into(out, y, inv, w, shared, topk)
        self.combine_fn = combine_fn

    def __call__(self, local2d: torch.Tensor) -> None:
        """local2d: this rank's packed down shard as [rows, H] (routed rows + its shared rows)."""
        if self.send.shape[0]:
            torch.index_select(local2d, 0, self.send_idx, out=self.send)
        _all_to_all_rows(self.recv[: self.recv.shape[0] - 1], self.send, self.out_splits, self.in_splits, self.group)
        sb = self.cp.shared_base[self.rank]
        shared = local2d[sb:sb + self.n] if sb >= 0 else None
        self.combine_fn(self.out[: self.n], self.recv, self.inv, self.w, shared, self.cp.topk)
        if self.gather_output:
            _all_gather(self.gathered.view(-1), self.out.view(-1), self.group)

    def full_output(self) -> torch.Tensor:
        """The combined [T, H] layer output from the all-gathered buffer (gather_output=True)."""
        parts = [self.gathered[r * max(self.pad, 1): r * max(self.pad, 1) + (t1 - t0)]
                 for r, (t0, t1) in enumerate(self.cp.token_range)]
        return torch.cat(parts, 0)


class EPCombineStep:
    """The second N > 1 step: EPLayerStep's compute (gate_up + down over this rank's row items; one
    chunk) followed by the token-owner exchange (CombineExchange) instead of the all-gather of every
    expert's down C."""

    def __init__(self, gate_up, down, world: int, rank: int, routing: TokenRouting, variant: Optional[int] = None,
                 group=None, shared: bool = True, gather_output: bool = True):
        self.ep = EPLayerStep(gate_up, down, world, rank, variant=variant, group=group, shared=shared, chunks=1)
        H = down.shapes[0].N
        if any(s.N != H for s in down.shapes):
            raise ValueError("the down problems must share N (= hidden)")
        self.cplan = ep_combine_plan(self.ep.plan, down.shapes, routing, shared)
        self.local2d = self.ep.parts[0][2][: sum(w.rows for w in self.ep.plan[rank]) * H].view(-1, H)
        self.xchg = CombineExchange(self.cplan, rank, H, self.local2d.device, gather_output=gather_output, group=group)
        self.flops_local = self.ep.flops_local

    def compute(self, stream: Optional[torch.cuda.Stream] = None) -> None:
        self.ep.compute(stream)

    def exchange(self, stream: Optional[torch.cuda.Stream] = None) -> None:
        with torch.cuda.stream(stream) if stream is not None else _null():
            self.xchg(self.local2d)

    def __call__(self, stream: torch.cuda.Stream) -> None:
        self.ep.compute(stream)
        self.exchange(stream)


class _null:
    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False


COMBINE_GBS = 6000.0  # mxmoe_moe_combine's measured streaming rate (6.5 TB/s at bs 8192)


def exchange_model(t_compute_ms: float, world: int, pad_elems: int, cplan: Optional[CombinePlan], H: int,
                   link_gbs: float = XGMI_LINK_GBS) -> dict:
    """Modelled N > 1 step of both exchanges from a rank's compute time (all in ms; links as in
    gather_ms_model):
      allgather:   north_star's form — every rank's per-expert down C all-gathered (EPLayerStep),
                   compute and gather pipelined in dist.choose_chunks chunks;
      combine:     the token-owner exchange (EPCombineStep) — all-to-all of routed rows to their
                   token's owner, the combine there, all-gather of the combined [T, H] output;
      combine_sharded: the same without the final all-gather (the output stays token-sharded, the
                   layout a data-parallel consumer of the layer reads)."""
    tg = gather_ms_model(2.0 * pad_elems * (world - 1), world, link_gbs)
    c = choose_chunks(t_compute_ms, tg)
    lo, hi = sorted((t_compute_ms, tg))
    out = {"allgather": {"MB_received": round(2.0 * pad_elems * (world - 1) / 1e6, 1), "gather_ms": round(tg, 4),
                         "chunks": c, "step_ms": round(hi + lo / c + (c - 1) * CHUNK_OVERHEAD_MS, 4)}}
    if cplan is not None:
        b = cplan.bytes_received(H)
        a2a = max(b["all_to_all"])
        ag = max(b["allgather_out"])
        n_max = max(t1 - t0 for t0, t1 in cplan.token_range)
        t_a2a = gather_ms_model(a2a, world, link_gbs)
        t_ag = gather_ms_model(ag, world, link_gbs)
        t_comb = n_max * H * 2 * (cplan.topk + 2) / (COMBINE_GBS * 1e9) * 1e3
        out["combine"] = {"a2a_MB_received": round(a2a / 1e6, 1), "allgather_out_MB_received": round(ag / 1e6, 1),
                          "a2a_ms": round(t_a2a, 4), "combine_ms": round(t_comb, 4), "allgather_out_ms": round(t_ag, 4),
                          "step_ms": round(t_compute_ms + t_a2a + t_comb + t_ag, 4)}
        out["combine_sharded"] = {"step_ms": round(t_compute_ms + t_a2a + t_comb, 4)}
    return out


def link_gbs_for_speedup(t1_ms: float, t_compute_ms: float, world: int, pad_elems: int, cplan: Optional[CombinePlan],
                         H: int, target: float = 3.5, forms=("allgather", "combine", "combine_sharded"),
                         hi_gbs: float = 10000.0) -> dict:
    """Per exchange form, the effective xGMI GB/s per link (and direction) at which exchange_model's
    step reaches ``target`` x the one-GPU layer time t1_ms; None where even an infinitely fast link
    cannot (compute + fixed costs alone miss the target). Bisection on the monotone step(link) —
    what a SCALE run has to show per link for north_star's >= 3.5x at 8 GPUs."""
    out = {}
    for form in forms:
        if form != "allgather" and cplan is None:
            continue

        def speedup(gbs: float) -> float:
            return t1_ms / exchange_model(t_compute_ms, world, pad_elems, cplan, H, link_gbs=gbs)[form]["step_ms"]

        if speedup(hi_gbs) < target:
            out[form] = None
            continue
        lo, hi = 1e-3, hi_gbs
        for _ in range(60):
            mid = (lo * hi) ** 0.5
            lo, hi = (mid, hi) if speedup(mid) < target else (lo, mid)
        out[form] = round(hi, 1)
    return out
