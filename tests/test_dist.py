"""Multi-process (gloo, world_size 2 and 4, CPU) tests of the multi-GPU partitioning + exchange."""
from __future__ import annotations

import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from mxmoe_amd.dist import allgather_outputs, ep_layer_chunks, ep_layer_plan, ep_scatter, ep_shard, ep_shard_elems, lpt_assign, nslice_plan
from mxmoe_amd.workload import load_workload, qwen2_layer11_workload


def _layer():
    return load_workload(qwen2_layer11_workload(8192, qstr="w8a8_g-1_sym"))["layer-11"]


def test_lpt_balance():
    owner = lpt_assign([10, 9, 8, 7, 6, 5, 4], 3)
    loads = [sum(c for c, o in zip([10, 9, 8, 7, 6, 5, 4], owner) if o == r) for r in range(3)]
    assert max(loads) - min(loads) <= 4


@pytest.mark.parametrize("world", [2, 4, 8])
def test_ep_shard_covers_each_expert_once(world):
    layer = _layer()
    seen = []
    per_rank = []
    for r in range(world):
        sh = ep_shard(layer, world, r)
        assert sh["gate_up"][-1].M == 8192  # replicated shared expert on local tokens
        per_rank.append(sum(p.flops for gg in sh for p in sh[gg]))
        seen += [p.N for p in sh["gate_up"][:-1]]
    assert len(seen) == 60
    single = sum(p.flops for gg in layer for p in layer[gg])
    assert max(per_rank) < 1.06 * single  # weak scaling: ~one layer of work per rank


@pytest.mark.parametrize("world", [2, 8])
def test_nslice_plan_splits_shared_expert(world):
    layer = _layer()["gate_up"]
    plan = nslice_plan(layer, world)
    covered = {}
    for work in plan:
        for w in work:
            covered.setdefault(w.problem, []).append((w.n0, w.n1))
    for i, s in enumerate(layer):
        spans = sorted(covered[i])
        assert spans[0][0] == 0 and spans[-1][1] == s.N
        assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))
        assert all((n1 - n0) % 256 == 0 or n1 == s.N for n0, n1 in spans)
    loads = [sum(2 * layer[w.problem].M * w.width * layer[w.problem].K for w in work) for work in plan]
    assert max(loads) / (sum(loads) / world) < 1.15  # the shared expert no longer caps the speedup at 2x


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from mxmoe_amd.workload import QShape

        shapes = [QShape([37, 512, 64]), QShape([5, 256, 64]), QShape([64, 1024, 64]), QShape([0, 256, 64])]
        plan = nslice_plan(shapes, world, slice_n=256, target_frac=0.3)
        # each rank "computes" its slices: value = 1000*problem + column, packed in work order
        parts = []
        for w in plan[rank]:
            M = shapes[w.problem].M
            cols = torch.arange(w.n0, w.n1, dtype=torch.float32)
            parts.append((1000.0 * w.problem + cols).expand(M, -1).reshape(-1))
        local = torch.cat(parts) if parts else torch.zeros(0)
        outs = [torch.full((max(s.M, 1), s.N), -1.0) for s in shapes]
        allgather_outputs(shapes, plan, local, outs)
        ok = all(torch.equal(outs[i][: s.M], (1000.0 * i + torch.arange(s.N, dtype=torch.float32)).expand(s.M, -1))
                 for i, s in enumerate(shapes))
        # the max-over-ranks timing reduction bench.py uses
        t = torch.tensor([float(rank + 1)], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        q.put((rank, ok, float(t.item())))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
def test_allgather_outputs_gloo(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in ps:
        p.join(timeout=60)
    assert all(ok for _, ok, _ in res)
    assert all(t == float(world) for _, _, t in res)


def _oracle_slice(A, B, sa, sb, M, w, K, bits):
    """Oracle output of columns [n0, n1) of one problem (test infrastructure)."""
    from oracle import oracle

    Bs = B[w.n0:w.n1]
    if bits == 16:
        return oracle.gg_f16(A, Bs, M, w.width, K)
    return oracle.gg_quant(A, Bs, sa, sb[w.n0:w.n1], M, w.width, K, bits)


def _layer_worker(rank, world, port, q):
    """Each rank computes its nslice_plan work list with the oracle, packs the C slices into one shard
    in work order and all-gathers; every rank then checks the reassembled layer against the oracle's
    full-layer C (bit-exact: column slicing does not change any output element's arithmetic)."""
    import numpy as np

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from tests._util import HostProblem
        from mxmoe_amd.groupgemm import FP16, W4A4, W8A8
        from mxmoe_amd.workload import QShape

        specs = [(37, 768, 128, W8A8), (5, 256, 256, W4A4), (70, 1024, 128, W8A8), (0, 256, 128, W4A4),
                 (19, 512, 64, FP16), (64, 1280, 256, W4A4)]  # last one: "shared expert", N-split
        hps = [HostProblem(M, N, K, qq, seed=900 + i, device="cpu") for i, (M, N, K, qq) in enumerate(specs)]
        shapes = [QShape([h.M, h.N, h.K], h.q.w_bits, h.q.a_bits, h.q.gsize, h.q.sym) for h in hps]
        plan = nslice_plan(shapes, world, slice_n=256, target_frac=0.5)
        parts = []
        for w in plan[rank]:
            h = hps[w.problem]
            c = _oracle_slice(h.A, h.B, h.sa, h.sb, h.M, w, h.K, 16 if not h.q.is_quant else h.q.a_bits)
            parts.append(torch.from_numpy(np.ascontiguousarray(c)).reshape(-1))
        local = torch.cat(parts) if parts else torch.zeros(0, dtype=torch.float16)
        outs = [torch.full((max(s.M, 1), s.N), float("nan"), dtype=torch.float16) for s in shapes]
        allgather_outputs(shapes, plan, local, outs)
        ok = all(np.array_equal(outs[i][: h.M].numpy().view(np.uint16), h.expected().view(np.uint16))
                 for i, h in enumerate(hps) if h.M)
        split = max(sum(1 for work in plan for w in work if w.problem == 5), 0)
        q.put((rank, ok, split))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2])
def test_nslice_layer_reassembles_oracle_output_gloo(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_layer_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = [q.get(timeout=300) for _ in range(world)]
    for p in ps:
        p.join(timeout=60)
    assert all(ok for _, ok, _ in res)
    assert all(split >= 2 for *_, split in res)  # the largest problem really was N-split across ranks


@pytest.mark.parametrize("world", [1, 2, 4, 8])
@pytest.mark.parametrize("model", ["qwen2", "ds2", "mixtral"])
def test_ep_layer_plan_covers_layer_and_balances(world, model):
    from mxmoe_amd.workload import model_workload

    if model == "qwen2":
        layer = _layer()
    else:
        layer = next(iter(load_workload(model_workload(model, 8192)).values()))
    gu, dn = layer["gate_up"], layer["down"]
    shared = model != "mixtral"
    plan = ep_layer_plan(gu, dn, world, shared=shared)
    rows = {}
    for items in plan:
        for w in items:
            rows.setdefault(w.problem, []).append((w.m0, w.m1))
    for i, s in enumerate(gu):
        if s.M == 0:
            assert i not in rows
            continue
        spans = sorted(rows[i])
        assert spans[0][0] == 0 and spans[-1][1] == s.M and all(a[1] == b[0] for a, b in zip(spans, spans[1:]))
        if not (shared and i == len(gu) - 1):
            assert len(spans) == 1  # a routed expert is never split: its gate_up output stays on its rank
        else:
            assert all(m0 % 64 == 0 for m0, _ in spans)
    loads = [sum(w.rows * (gu[w.problem].N * gu[w.problem].K + dn[w.problem].N * dn[w.problem].K) for w in items)
             for items in plan]
    if shared:  # the shared expert's rows even out the routed experts' LPT remainder
        assert max(loads) / (sum(loads) / world) < 1.03
    assert sum(ep_shard_elems(dn, items) for items in plan) == sum(s.M * s.N for s in dn)


def _ep_worker(rank, world, port, q):
    """Each rank computes the down outputs of its ep_layer_plan row items with the oracle, packs them
    in work order, all-gathers, scatters, and checks the whole layer output against the oracle's
    full-problem C (bit-exact: a row slice does not change any output element's arithmetic)."""
    import numpy as np

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from oracle import oracle
        from tests._util import HostProblem
        from mxmoe_amd.groupgemm import FP16, W4A4, W8A8
        from mxmoe_amd.workload import QShape

        specs = [(37, 256, 128, W8A8), (5, 256, 256, W4A4), (70, 128, 128, W8A8), (0, 256, 128, W4A4),
                 (19, 256, 64, FP16), (640, 256, 256, W4A4)]  # last one: the shared expert, row-split
        hps = [HostProblem(M, N, K, qq, seed=700 + i, device="cpu") for i, (M, N, K, qq) in enumerate(specs)]
        shapes = [QShape([h.M, h.N, h.K], h.q.w_bits, h.q.a_bits, h.q.gsize, h.q.sym) for h in hps]
        plan = ep_layer_plan(shapes, shapes, world)
        pad = max(ep_shard_elems(shapes, w) for w in plan)
        parts = []
        for w in plan[rank]:
            h = hps[w.problem]
            K = h.K
            if h.q.is_quant:
                c = oracle.gg_quant(h.A[w.m0:w.m1], h.B, h.sa[w.m0:w.m1], h.sb, w.rows, h.N, K, h.q.a_bits)
            else:
                c = oracle.gg_f16(h.A[w.m0:w.m1], h.B, w.rows, h.N, K)
            parts.append(torch.from_numpy(np.ascontiguousarray(c)).reshape(-1))
        local = torch.zeros(pad, dtype=torch.float16)
        if parts:
            cat = torch.cat(parts)
            local[:cat.numel()] = cat
        gathered = torch.empty(world * pad, dtype=torch.float16)
        dist.all_gather_into_tensor(gathered, local)
        outs = [torch.full((max(s.M, 1), s.N), float("nan"), dtype=torch.float16) for s in shapes]
        ep_scatter(shapes, plan, gathered, pad, outs)
        ok = all(np.array_equal(outs[i][: h.M].numpy().view(np.uint16), h.expected().view(np.uint16))
                 for i, h in enumerate(hps) if h.M)
        split = sum(1 for items in plan for w in items if w.problem == 5)
        q.put((rank, ok, split))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2])
def test_ep_layer_reassembles_oracle_output_gloo(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_ep_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = [q.get(timeout=300) for _ in range(world)]
    for p in ps:
        p.join(timeout=60)
    assert all(ok for _, ok, _ in res), res
    assert all(split == world for *_, split in res)  # the shared expert's rows were split over the ranks


@pytest.mark.parametrize("chunks", [1, 2, 3])
def test_ep_layer_chunks_partition_each_rank(chunks):
    layer = _layer()
    gu, dn = layer["gate_up"], layer["down"]
    plan = ep_layer_plan(gu, dn, 8)
    cps = ep_layer_chunks(plan, gu, dn, chunks)
    assert len(cps) == chunks
    for r, items in enumerate(plan):
        rows = {}
        for cp in cps:
            for w in cp[r]:
                rows.setdefault(w.problem, []).append((w.m0, w.m1))
        assert sorted(rows) == sorted(w.problem for w in items)
        for w in items:
            spans = sorted(rows[w.problem])
            assert spans[0][0] == w.m0 and spans[-1][1] == w.m1 and all(a[1] == b[0] for a, b in zip(spans, spans[1:]))
        if chunks > 1:
            loads = [sum(w.rows * (gu[w.problem].N * gu[w.problem].K + dn[w.problem].N * dn[w.problem].K) for w in cp[r])
                     for cp in cps]
            assert max(loads) < 1.35 * sum(loads) / chunks


def test_choose_chunks_model():
    from mxmoe_amd.dist import choose_chunks, gather_ms_model

    assert choose_chunks(0.5, 0.0) == 1  # nothing to hide
    assert choose_chunks(0.0, 0.3) == 1
    # compute and gather comparable: pipelining pays, more chunks while the overhead stays small
    assert choose_chunks(0.19, 0.33) > 1
    assert choose_chunks(0.19, 0.33, overhead_ms=1.0) == 1
    assert choose_chunks(1.0, 1.0) >= choose_chunks(0.2, 0.2)
    assert 1 <= choose_chunks(5.0, 5.0) <= 8
    # qwen2_moe layer 11 at N = 8: 147 MB received per rank over 7 links
    t = gather_ms_model(147e6, 8)
    assert 0.2 < t < 0.5 and gather_ms_model(147e6, 1) == 0.0
    assert gather_ms_model(84e6, 2) > gather_ms_model(147e6, 8)


# ------------------------------------------------------------------ combine before the exchange

def _combine_layer(seed=0):
    """A small MoE down call: 6 routed experts (one empty) + the shared expert over T = 96 tokens,
    top-2 routing with some dropped choices, hidden H = 128, mixed quant types."""
    from mxmoe_amd.dist import synthetic_routing
    from mxmoe_amd.groupgemm import FP16, W4A4, W8A8

    T, topk, H = 96, 2, 128
    counts = [30, 5, 41, 0, 19, 64]
    qs = [W8A8, W4A4, W8A8, W4A4, FP16, W4A4, W8A8]  # last: shared
    specs = [(c, H, 64, q) for c, q in zip(counts, qs)] + [(T, H, 128, qs[-1])]
    return specs, synthetic_routing(counts, T, topk, seed=seed), T, topk, H


def test_ep_combine_plan_routes_every_row_once():
    import numpy as np

    from mxmoe_amd.dist import ep_combine_plan, synthetic_routing
    from mxmoe_amd.workload import QShape

    layer = _layer()
    dn = layer["down"]
    T = dn[-1].M
    routing = synthetic_routing([s.M for s in dn[:-1]], T, 4, seed=3)
    assert (routing.topk_ids >= 0).sum() == sum(s.M for s in dn[:-1])
    for world in (1, 2, 4, 8):
        plan = ep_layer_plan(layer["gate_up"], dn, world)
        cp = ep_combine_plan(plan, dn, routing)
        assert cp.token_range[0][0] == 0 and cp.token_range[-1][1] == T
        # every routed row is sent exactly once, and every owned (token, choice) reads a distinct row
        sent = sum(len(cp.send_rows[s][d]) for s in range(world) for d in range(world))
        assert sent == sum(s.M for s in dn[:-1])
        for d in range(world):
            R = cp.recv_rows[d]
            real = cp.inv_local[d][cp.inv_local[d] < R]
            assert len(np.unique(real)) == len(real) and (cp.inv_local[d] <= R).all()
        b = cp.bytes_received(2048)
        if world == 8:  # the token-owner exchange moves far fewer bytes than the per-expert all-gather
            pad = max(ep_shard_elems(dn, items) for items in plan)
            assert max(b["all_to_all"]) + max(b["allgather_out"]) < 0.4 * 2 * pad * (world - 1)
    _ = QShape


def _combine_worker(rank, world, port, q):
    """Each rank computes the down outputs of its ep_layer_plan items with the oracle, runs the
    token-owner exchange (CombineExchange: index_select, all_to_all_single, the oracle combine as
    the local combine, all-gather of the combined rows) and checks the [T, H] layer output against
    the oracle's one-process combine of the whole layer, bit for bit."""
    import numpy as np

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from oracle import moe_ref
        from tests._util import HostProblem
        from mxmoe_amd.dist import CombineExchange, ep_combine_plan
        from mxmoe_amd.workload import QShape

        specs, routing, T, topk, H = _combine_layer()
        hps = [HostProblem(M, N, K, qq, seed=500 + i, device="cpu") for i, (M, N, K, qq) in enumerate(specs)]
        shapes = [QShape([h.M, h.N, h.K], h.q.w_bits, h.q.a_bits, h.q.gsize, h.q.sym) for h in hps]
        full = [h.expected() if h.M else np.zeros((0, H), np.float16) for h in hps]
        plan = ep_layer_plan(shapes, shapes, world)
        cp = ep_combine_plan(plan, shapes, routing)
        rows = [full[w.problem][w.m0:w.m1] for w in plan[rank]]  # this rank's "down GroupGEMM" output
        local = torch.from_numpy(np.ascontiguousarray(np.concatenate(rows) if rows else np.zeros((0, H), np.float16)))

        def oracle_combine(out, y, inv, w, shared, k):
            if out.shape[0]:
                out.copy_(torch.from_numpy(moe_ref.combine(y.numpy(), inv.numpy(), w.numpy(), k,
                                                           None if shared is None else shared.numpy())))

        x = CombineExchange(cp, rank, H, "cpu", combine_fn=oracle_combine)
        x(local)
        got = x.full_output().numpy()
        # the reference: the whole layer combined in one process (y in slot order + a zero row)
        _, _, inv, counts, _ = routing.slots()
        y = np.concatenate([full[e] for e in range(len(counts))] + [np.zeros((1, H), np.float16)])
        inv_ref = np.minimum(inv, y.shape[0] - 1).astype(np.int32)
        ref = moe_ref.combine(y, inv_ref, routing.weights, topk, full[-1])
        q.put((rank, bool(np.array_equal(got.view(np.uint16), ref.view(np.uint16))), cp.recv_rows[rank]))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_ep_combine_exchange_reassembles_oracle_combine_gloo(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_combine_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = [q.get(timeout=300) for _ in range(world)]
    for p in ps:
        p.join(timeout=60)
    assert all(ok for _, ok, _ in res), res
    assert sum(r for *_, r in res) > 0


def test_exchange_model_token_owner_beats_allgather_at_8():
    """with the round-4 per-rank compute (0.168 ms at N = 8 against T1 = 1.053 ms)
    the modelled token-owner exchange reaches >= 3.5x where north_star's per-expert all-gather stays
    near 2.5x."""
    from mxmoe_amd.dist import ep_combine_plan, exchange_model, synthetic_routing

    layer = _layer()
    gu, dn = layer["gate_up"], layer["down"]
    routing = synthetic_routing([s.M for s in dn[:-1]], dn[-1].M, 4)
    plan = ep_layer_plan(gu, dn, 8)
    pad = max(ep_shard_elems(dn, it) for it in plan)
    m = exchange_model(0.168, 8, pad, ep_combine_plan(plan, dn, routing), 2048)
    assert 1.053 / m["allgather"]["step_ms"] < 3.0
    assert 1.053 / m["combine"]["step_ms"] >= 3.5
    assert m["combine_sharded"]["step_ms"] < m["combine"]["step_ms"] < m["allgather"]["step_ms"]
    assert m["combine"]["a2a_MB_received"] + m["combine"]["allgather_out_MB_received"] < 0.35 * m["allgather"]["MB_received"]


class _FakeDeviceTensor:
    """Stands in for a CUDA tensor on the CPU-only host: .is_cuda is True and any host staging
    (.cpu()) fails the test, so the RCCL branch must pass it to the collective untouched."""

    is_cuda = True

    def cpu(self):
        raise AssertionError("device tensor staged through host memory under a non-gloo backend")


@pytest.mark.parametrize("backend", ["nccl", "mpi"])
def test_collectives_pass_device_tensors_straight_to_rccl(monkeypatch, backend):
    """under any backend but gloo (RCCL is torch's "nccl" on ROCm) _all_gather and
    _all_to_all_rows hand the device tensors themselves to the collective — no host round trip; under
    gloo with device tensors (the one-GPU rehearsal) they stage through host memory."""
    import mxmoe_amd.dist as md

    calls = []
    monkeypatch.setattr(dist, "get_backend", lambda group=None: backend)
    monkeypatch.setattr(dist, "all_gather_into_tensor", lambda out, inp, group=None: calls.append(("ag", out, inp)))
    monkeypatch.setattr(dist, "all_to_all_single",
                        lambda out, inp, osp, isp, group=None: calls.append(("a2a", out, inp, osp, isp)))
    out, inp = _FakeDeviceTensor(), _FakeDeviceTensor()
    md._all_gather(out, inp)
    md._all_to_all_rows(out, inp, [1, 2], [2, 1])
    assert calls == [("ag", out, inp), ("a2a", out, inp, [1, 2], [2, 1])]


def test_collectives_stage_device_tensors_under_gloo(monkeypatch):
    """The gloo branch (device tensors, one-GPU rehearsal): the collective sees host tensors and the
    result is copied back into the device output."""
    import mxmoe_amd.dist as md

    seen = []

    class Dev:
        is_cuda = True

        def __init__(self, t):
            self.t = t
            self.shape = t.shape
            self.dtype = t.dtype

        def numel(self):
            return self.t.numel()

        def cpu(self):
            return self.t.clone()

        def copy_(self, src):
            self.t.copy_(src)

    def ag(out, inp, group=None):
        seen.append(type(inp))
        out.copy_(torch.cat([inp, inp]))

    def a2a(out, inp, osp, isp, group=None):
        seen.append(type(inp))
        out.copy_(inp)

    monkeypatch.setattr(dist, "get_backend", lambda group=None: "gloo")
    monkeypatch.setattr(dist, "all_gather_into_tensor", ag)
    monkeypatch.setattr(dist, "all_to_all_single", a2a)
    out, inp = Dev(torch.zeros(4)), Dev(torch.tensor([1.0, 2.0]))
    md._all_gather(out, inp)
    assert out.t.tolist() == [1.0, 2.0, 1.0, 2.0]
    rows = Dev(torch.zeros(2, 3))
    md._all_to_all_rows(rows, Dev(torch.ones(2, 3)), [2], [2])
    assert rows.t.sum().item() == 6.0
    assert seen == [torch.Tensor, torch.Tensor]


def test_link_rate_for_3p5x_at_8():
    """the per-link xGMI rate each exchange needs for 3.5x at N = 8 (round-4 per-rank
    compute 0.168 ms, T1 1.053 ms): the modelled step at the solved rate sits on the target, the
    per-expert all-gather needs several times the token-owner exchange's rate, and the token-sharded
    output the least."""
    from mxmoe_amd.dist import ep_combine_plan, exchange_model, link_gbs_for_speedup, synthetic_routing

    layer = _layer()
    gu, dn = layer["gate_up"], layer["down"]
    routing = synthetic_routing([s.M for s in dn[:-1]], dn[-1].M, 4)
    plan = ep_layer_plan(gu, dn, 8)
    pad = max(ep_shard_elems(dn, it) for it in plan)
    cp = ep_combine_plan(plan, dn, routing)
    need = link_gbs_for_speedup(1.053, 0.168, 8, pad, cp, 2048)
    assert need["combine_sharded"] < need["combine"] < need["allgather"]
    for form, gbs in need.items():
        step = exchange_model(0.168, 8, pad, cp, 2048, link_gbs=gbs)[form]["step_ms"]
        assert 3.45 <= 1.053 / step <= 3.6, (form, gbs, step)
    # below the compute bound no link rate suffices
    assert link_gbs_for_speedup(1.053, 0.32, 8, pad, cp, 2048)["combine"] is None
