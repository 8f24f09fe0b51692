"""The gate_up GroupGEMM's fused SiLU·mul epilogue (MXMOE_GG_EPI_SILU_MUL, include/mxmoe_gg.h) and
the slot quantiser behind it (mxmoe_moe_quant_slots, include/mxmoe_moe.h) — §8(f) rank 2, the MoE
layer's silu_mul_then_quant (ref_bind.cu:595-757) folded into the GEMM that produces its input.

CPU: the gate / up interleave, the ABI's validation of the flag (types, N % 32, variants, AUTO
handing small fused calls to the small-batch kernel, whose fp16 / w8a8 / w4a4 bodies carry it). GPU: fused outputs against the unfused call + the
oracle SiLU (1 fp16 ulp, as the MoE plumbing tests), the slot quantiser against silu_mul_quant bit
for bit, and MoEFFN with and without fusion returning bit-identical layers.
"""
from __future__ import annotations

import numpy as np
import pytest
import torch

from mxmoe_amd import _native as nat
from mxmoe_amd import moe
from mxmoe_amd.groupgemm import FP16, W4A4, W4A4_G128, W8A8, GroupGemm, Problem, QParams, interleave_gate_up
from oracle import moe_ref

DEV = "cuda"


def test_interleave_gate_up_blocks():
    n = 64
    w = torch.arange(2 * n).view(2 * n, 1).repeat(1, 3)
    s = torch.arange(2 * n, dtype=torch.float32)
    w2, s2 = interleave_gate_up(w, s)
    rows = w2[:, 0].tolist()
    for b in range(n // 16):
        assert rows[32 * b: 32 * b + 16] == list(range(16 * b, 16 * b + 16))  # gate block b
        assert rows[32 * b + 16: 32 * b + 32] == list(range(n + 16 * b, n + 16 * b + 16))  # up block b
    assert torch.equal(s2, w2[:, 0].float())
    with pytest.raises(ValueError):
        interleave_gate_up(torch.zeros(48, 4))


def _cp(M, N, K, q, silu=True, ldc=0):
    return nat.GGProblemC(A=16, B=16, scale_a=16, scale_b=16, C=16, M=M, N=N, K=K, a_bits=q.a_bits, w_bits=q.w_bits,
                          gsize=q.gsize, sym=int(q.sym), fmt=q.fmt_code | (nat.EPI_SILU_MUL if silu else 0), lda=0,
                          ldb=0, ldc=ldc)


def _arr(*ps):
    return (nat.GGProblemC * len(ps))(*ps)


def test_flag_validation():
    names = [ln.split()[1] for ln in nat.list_variants()]
    wo3, v2x = names.index("wo3_64x256_w8_3wg"), names.index("v2x_256x256_w8_b3_buf_spread_edma")
    ok = _arr(_cp(300, 512, 256, W8A8), _cp(70, 2816, 2048, FP16), _cp(5, 512, 256, W4A4))
    assert nat.workspace_size(ok, 3, v2x) > 0
    with pytest.raises(nat.GGError, match="N % 32"):
        nat.workspace_size(_arr(_cp(64, 528, 256, W8A8)), 1, v2x)
    with pytest.raises(nat.GGError, match="SiLU epilogue needs"):
        nat.workspace_size(_arr(_cp(64, 512, 256, W4A4_G128)), 1, v2x)
    with pytest.raises(nat.GGError, match="SiLU epilogue needs"):
        nat.workspace_size(_arr(_cp(64, 512, 256, QParams(16, 4, 128, False))), 1, v2x)
    assert nat.workspace_size(_arr(_cp(64, 512, 256, W8A8), _cp(30, 512, 256, W4A4), _cp(9, 256, 128, FP16)), 3, wo3) > 0
    # weight-only problems carry it on wo3 only (its WO_SILU builds)
    assert nat.workspace_size(_arr(_cp(64, 512, 256, QParams(16, 4, 128, False)), _cp(9, 256, 128, W8A8)), 2, wo3) > 0
    with pytest.raises(nat.GGError, match="ldc"):
        nat.workspace_size(_arr(_cp(64, 512, 256, W8A8, ldc=200)), 1, v2x)
    assert nat.workspace_size(_arr(_cp(64, 512, 256, W8A8, ldc=256)), 1, v2x) > 0  # ldc >= N / 2 suffices
    bad = _cp(64, 512, 256, W8A8)
    bad.fmt |= 0x200
    with pytest.raises(nat.GGError, match="unknown fmt flags"):
        nat.workspace_size(_arr(bad), 1, v2x)
    # small batch: AUTO takes wo3 for the plain call and for the fused one alike (round 6)
    small = [_cp(30, 2816, 2048, W8A8, silu=False) for _ in range(8)]
    assert names[nat.resolve_variant(_arr(*small), 8)] == "wo3_64x256_w8_3wg"
    fused = [_cp(30, 2816, 2048, W8A8) for _ in range(8)]
    assert names[nat.resolve_variant(_arr(*fused), 8)] == "wo3_64x256_w8_3wg"
    # w4a4-only calls keep their kernel (v3 has the epilogue too)
    assert names[nat.resolve_variant(_arr(_cp(4096, 2816, 2048, W4A4)), 1)] == "v3_256x128_w4_dma_ring3_2wg"


# ------------------------------------------------------------------------------------------ GPU
@pytest.fixture()
def gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    nat.lib()


def _gate_up_problem(M, Nh, K, q, seed, ldc=0):
    """Unfused and fused problems over the same quantised operands (B [2 Nh, K] = [gate; up])."""
    from mxmoe_amd.quantize import pack_wxax, quant_rtn_sym

    g = torch.Generator().manual_seed(seed)
    a = ((torch.rand(M, K, generator=g) * 2 - 1)).half().to(DEV)
    b = ((torch.rand(2 * Nh, K, generator=g) * 2 - 1) * 0.25).half().to(DEV)
    if q.is_quant:
        qa, sa = quant_rtn_sym(a, q.a_bits, -1)
        qb, sb = quant_rtn_sym(b, q.w_bits, -1)
        A, B = pack_wxax(qa, q.a_bits), pack_wxax(qb, q.w_bits)
    else:
        A, B, sa, sb = a, b, None, None
    C = torch.empty(max(M, 1), 2 * Nh, dtype=torch.float16, device=DEV)
    plain = Problem(A=A, B=B, C=C, M=M, N=2 * Nh, K=K, q=q, scale_a=sa, scale_b=sb)
    Bi, sbi = interleave_gate_up(B, sb)
    Cf = torch.full((max(M, 1), ldc or Nh), float("nan"), dtype=torch.float16, device=DEV)
    fused = Problem(A=A, B=Bi, C=Cf, M=M, N=2 * Nh, K=K, q=q, scale_a=sa, scale_b=sbi, silu=True, ldc=ldc)
    return plain, fused


@pytest.mark.gpu
@pytest.mark.parametrize("q", [FP16, W8A8, W4A4], ids=["fp16", "w8a8", "w4a4"])
@pytest.mark.parametrize("vname", ["v2x_256x256_w8_b3_buf_spread_edma", "v3_256x128_w4_dma_ring3_2wg", "wo3_64x256_w8_3wg",
                                   "auto"])
def test_fused_epilogue_matches_unfused_plus_silu(gpu, q, vname):
    names = [ln.split()[1] for ln in nat.list_variants()]
    variant = None if vname == "auto" else names.index(vname)
    shapes = [(300, 256, 256), (70, 1408, 512), (1, 128, 128), (129, 512, 384), (513, 272, 256), (0, 256, 256),
              (64, 128, 1024), (200, 384, 256)]
    pairs = [_gate_up_problem(M, Nh, K, q, seed=40 + i, ldc=(Nh + 24 if i == 7 else 0))
             for i, (M, Nh, K) in enumerate(shapes)]
    GroupGemm([p for p, _ in pairs], variant=variant).launch()
    gg = GroupGemm([f for _, f in pairs], variant=variant)
    gg.launch()
    torch.cuda.synchronize()
    for (p, f), (M, Nh, K) in zip(pairs, shapes):
        if M == 0:
            continue
        ref = moe_ref.silu_mul(p.C[:M].cpu().numpy())
        out = f.C[:M, :Nh].cpu().numpy()
        assert np.isfinite(out).all()
        d = np.abs(out.view(np.uint16).astype(np.int32) - ref.view(np.uint16).astype(np.int32))
        same_sign = (np.signbit(out) == np.signbit(ref)) | (out == 0) | (ref == 0)
        assert same_sign.all() and (d <= 1).all(), f"{q.qcfg} M={M} Nh={Nh} K={K}: {int((d > 1).sum())} outputs > 1 ulp"
        if f.C.shape[1] > Nh:  # strided C: the columns past N / 2 untouched
            assert torch.isnan(f.C[:M, Nh:]).all()


@pytest.mark.gpu
def test_quant_slots_equals_silu_mul_quant(gpu):
    """quant_slots(act) == silu_mul_quant(gate_up) when act is silu_mul_quant's own fp16 activation."""
    T, topk, E, N, Ns = 300, 4, 8, 384, 1024
    g = torch.Generator().manual_seed(5)
    logits = torch.rand(T, E, generator=g)
    ids = torch.topk(logits, topk, dim=1).indices.to(torch.int32).to(DEV)
    r = moe.route(ids, E)
    routed = ((torch.rand(T * topk, 2 * N, generator=g) * 2 - 1) * 4).half().to(DEV)
    shared = ((torch.rand(T, 2 * Ns, generator=g) * 2 - 1) * 4).half().to(DEV)
    fp16 = [moe.ACT_FP16] * (E + 1)
    act = moe.silu_mul_quant(routed, shared, r, fp16)
    act_r = torch.empty(T * topk, N, dtype=torch.float16, device=DEV)
    for e, s in enumerate(act.segs[:E]):
        if s.rows:
            act_r[s.first_slot:s.first_slot + s.rows] = act.A(e).view(torch.float16).view(s.rows, N)
    act_s = act.A(E).view(torch.float16).view(T, Ns).clone()
    for tags in ([moe.ACT_INT8] * (E + 1), [moe.ACT_INT4, moe.ACT_INT8] * (E // 2) + [moe.ACT_INT4],
                 [moe.ACT_INT4_G128] * E + [moe.ACT_INT8]):
        a = moe.silu_mul_quant(routed, shared, r, tags)
        b = moe.silu_mul_quant(act_r, act_s, r, tags, activated=True)
        # the interleaved-input pass on the same values with gate / up columns in alternating
        # 16-column blocks (the fused layout through the plain epilogue)
        c = moe.silu_mul_quant(interleave_gate_up(routed.t())[0].t().contiguous(),
                               interleave_gate_up(shared.t())[0].t().contiguous(), r, tags, interleaved=True)
        torch.cuda.synchronize()
        assert torch.equal(a.out, b.out) and torch.equal(a.scales, b.scales), tags
        assert torch.equal(a.out, c.out) and torch.equal(a.scales, c.scales), tags


@pytest.mark.gpu
@pytest.mark.parametrize("T,override,variant", [(60, None, "wo3_64x256_w8_3wg"), (60, "interleaved", "wo3_64x256_w8_3wg"),
                                               (200, None, None), (2048, None, None)])
def test_moe_ffn_fused_equals_unfused(gpu, T, override, variant):
    """A fused-layout layer equals the plain one bit for bit; at T = 60 the gate_up call runs on wo3
    (its fused epilogue since round 6), and with the "interleaved" override the interleaved weights
    go through the plain epilogue and the interleaved-input SiLU pass (mxmoe_moe_silu_mul_quant_il)."""
    topk, E, H, N, Ns = 4, 6, 256, 384, 768
    g = torch.Generator().manual_seed(21)
    gate_up = [((torch.rand(2 * N, H, generator=g) * 2 - 1) * 0.2).half() for _ in range(E)]
    gate_up.append(((torch.rand(2 * Ns, H, generator=g) * 2 - 1) * 0.2).half())
    down = [((torch.rand(H, N, generator=g) * 2 - 1) * 0.2).half() for _ in range(E)]
    down.append(((torch.rand(H, Ns, generator=g) * 2 - 1) * 0.2).half())
    qcfg = [(W8A8, W8A8), (W4A4, W8A8), (FP16, FP16), (W8A8, W4A4), (W4A4, W4A4_G128), (W8A8, FP16), (W4A4, W8A8)]
    gu, dn = [w.to(DEV) for w in gate_up], [w.to(DEV) for w in down]
    plain = moe.MoEFFN(gu, dn, qcfg, num_routed=E, fuse_silu=False)
    fused = moe.MoEFFN(gu, dn, qcfg, num_routed=E)  # (default: fused when every gate_up qcfg allows)
    assert fused.fuse_silu
    fused.gate_up_mode = override
    mode = override or "fused"
    logits = torch.rand(T, E, generator=g)
    ids = torch.topk(logits, topk, dim=1).indices.to(torch.int32).to(DEV)
    wts = torch.softmax(torch.rand(T, topk, generator=g), dim=1).to(DEV)
    h = ((torch.rand(T, H, generator=g) * 2 - 1) * 3).half().to(DEV)
    o1, m1 = plain.forward(h, ids, wts, return_intermediates=True)
    o2, m2 = fused.forward(h, ids, wts, return_intermediates=True)
    torch.cuda.synchronize()
    assert torch.equal(m1["a2"].out, m2["a2"].out) and torch.equal(m1["a2"].scales, m2["a2"].scales)
    assert torch.equal(o1.view(torch.int16), o2.view(torch.int16))
    step = moe.PlannedForward(fused, h, ids, wts)
    assert step.mode == mode
    if variant:
        assert [ln.split()[1] for ln in nat.list_variants()][step.g1.variant] == variant
    with pytest.raises(ValueError, match="fuse_silu"):
        moe.MoEFFN(gu, dn, [(W4A4_G128, W8A8)] + qcfg[1:], num_routed=E, fuse_silu=True)


@pytest.mark.gpu
def test_planned_forward_graph_replay(gpu):
    """moe.PlannedForward (every launch pre-planned: quant_act, fused gate_up, quant_slots, down,
    combine) captured into one HIP graph: replays return the eager step's output bit for bit."""
    T, topk, E, H, N, Ns = 512, 4, 6, 256, 384, 768
    g = torch.Generator().manual_seed(31)
    gate_up = [((torch.rand(2 * N, H, generator=g) * 2 - 1) * 0.2).half().to(DEV) for _ in range(E)]
    gate_up.append(((torch.rand(2 * Ns, H, generator=g) * 2 - 1) * 0.2).half().to(DEV))
    down = [((torch.rand(H, N, generator=g) * 2 - 1) * 0.2).half().to(DEV) for _ in range(E)]
    down.append(((torch.rand(H, Ns, generator=g) * 2 - 1) * 0.2).half().to(DEV))
    qcfg = [(W8A8, W8A8), (W4A4, W8A8), (FP16, FP16), (W8A8, W4A4), (W4A4, W4A4), (W8A8, FP16), (W4A4, W8A8)]
    layer = moe.MoEFFN(gate_up, down, qcfg, num_routed=E, fuse_silu=True)
    ids = torch.topk(torch.rand(T, E, generator=g), topk, dim=1).indices.to(torch.int32).to(DEV)
    wts = torch.softmax(torch.rand(T, topk, generator=g), dim=1).to(DEV)
    h = ((torch.rand(T, H, generator=g) * 2 - 1) * 3).half().to(DEV)
    step = moe.PlannedForward(layer, h, ids, wts)
    eager = step().clone()
    ref = layer.forward(h, ids, wts)
    torch.cuda.synchronize()
    assert torch.equal(eager.view(torch.int16), ref.view(torch.int16))
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.stream(s):
        step()  # warm the stream
        torch.cuda.synchronize()
        step.out.fill_(float("nan"))
        with torch.cuda.graph(graph, stream=s):
            step()
    for _ in range(2):
        step.out.fill_(float("nan"))
        graph.replay()
        torch.cuda.synchronize()
        assert torch.equal(step.out.view(torch.int16), eager.view(torch.int16))


WO_QS = [QParams(16, 4, -1, False), QParams(16, 4, 128, False), QParams(16, 4, 128, True), QParams(16, 8, -1, False),
         QParams(16, 2, 128, False)]


def _wo_gate_up_problem(M, Nh, K, q, seed, ldc=0):
    """Weight-only unfused / fused problems over the same weights: the fused B is the gate_up weight
    interleaved BEFORE quantisation (per-row groups commute with the row order, as MoEFFN does)."""
    from mxmoe_amd.quantize import pack_weightonly_mi355x, quant_weightonly

    g = torch.Generator().manual_seed(seed)
    a = ((torch.rand(M, K, generator=g) * 2 - 1)).half().to(DEV)
    w = ((torch.rand(2 * Nh, K, generator=g) * 2 - 1) * 0.25).half().to(DEV)

    def packed(wt):
        codes, sz = quant_weightonly(wt, q.w_bits, q.gsize, q.sym)
        return pack_weightonly_mi355x(codes, q.w_bits), sz

    B, sz = packed(w)
    Bi, szi = packed(interleave_gate_up(w)[0])
    C = torch.empty(max(M, 1), 2 * Nh, dtype=torch.float16, device=DEV)
    plain = Problem(A=a, B=B, C=C, M=M, N=2 * Nh, K=K, q=q, scale_b=sz)
    Cf = torch.full((max(M, 1), ldc or Nh), float("nan"), dtype=torch.float16, device=DEV)
    fused = Problem(A=a, B=Bi, C=Cf, M=M, N=2 * Nh, K=K, q=q, scale_b=szi, silu=True, ldc=ldc)
    return plain, fused


def _check_fused(pairs, shapes):
    for (p, f), (M, Nh, K) in zip(pairs, shapes):
        if M == 0:
            continue
        ref = moe_ref.silu_mul(p.C[:M].cpu().numpy())
        out = f.C[:M, :Nh].cpu().numpy()
        assert np.isfinite(out).all()
        d = np.abs(out.view(np.uint16).astype(np.int32) - ref.view(np.uint16).astype(np.int32))
        same_sign = (np.signbit(out) == np.signbit(ref)) | (out == 0) | (ref == 0)
        assert same_sign.all() and (d <= 1).all(), f"{p.q.qcfg} M={M} Nh={Nh} K={K}: {int((d > 1).sum())} outputs > 1 ulp"
        if f.C.shape[1] > Nh:
            assert torch.isnan(f.C[:M, Nh:]).all()


@pytest.mark.gpu
@pytest.mark.parametrize("q", WO_QS, ids=[q.qcfg for q in WO_QS])
def test_fused_epilogue_weight_only_on_wo3(gpu, q):
    """Weight-only gate_up problems through the small-batch kernel's WO_SILU build (round 6): the
    fused outputs within 1 fp16 ulp of the oracle SiLU of the unfused call's outputs; edge shapes, a
    strided C, an empty problem, and a w8a8 problem with the flag in the same launch."""
    names = [ln.split()[1] for ln in nat.list_variants()]
    wo3 = names.index("wo3_64x256_w8_3wg")
    shapes = [(35, 256, 256), (70, 1408, 512), (1, 128, 128), (129, 512, 384), (0, 256, 256), (64, 128, 1024),
              (200, 384, 256)]
    pairs = [_wo_gate_up_problem(M, Nh, K, q, seed=60 + i, ldc=(Nh + 24 if i == 6 else 0))
             for i, (M, Nh, K) in enumerate(shapes)]
    pairs.append(_gate_up_problem(48, 256, 512, W8A8, seed=99))
    shapes.append((48, 256, 512))
    GroupGemm([p for p, _ in pairs], variant=wo3).launch()
    gg = GroupGemm([f for _, f in pairs])  # AUTO: the small-batch kernel, with the flag
    assert names[gg.variant] == "wo3_64x256_w8_3wg"
    assert gg.info.qtype_mask & (1 << 16)
    gg.launch()
    torch.cuda.synchronize()
    _check_fused(pairs, shapes)
    with pytest.raises(nat.GGError, match="SiLU epilogue needs"):  # the large-batch kernel has no WO_SILU tile
        GroupGemm([pairs[0][1]], variant=names.index("v2x_256x256_w8_b3_buf_spread_edma"))


@pytest.mark.gpu
@pytest.mark.parametrize("T,mode", [(60, "fused"), (2048, "interleaved")])
def test_moe_ffn_weight_only_fused_equals_unfused(gpu, T, mode):
    """The reference's small-batch MoE scheme (w4a16 experts beside w8a8, hz_fused.cuh:14-125) with
    the fused layout: bit-identical to the unfused layer; at T = 60 the gate_up call runs wo3's
    WO_SILU build, at T = 2048 the large-batch kernel (no weight-only SiLU tile) takes the
    interleaved form."""
    topk, E, H, N, Ns = 4, 6, 256, 384, 768
    g = torch.Generator().manual_seed(23)
    gate_up = [((torch.rand(2 * N, H, generator=g) * 2 - 1) * 0.2).half() for _ in range(E)]
    gate_up.append(((torch.rand(2 * Ns, H, generator=g) * 2 - 1) * 0.2).half())
    down = [((torch.rand(H, N, generator=g) * 2 - 1) * 0.2).half() for _ in range(E)]
    down.append(((torch.rand(H, Ns, generator=g) * 2 - 1) * 0.2).half())
    w4a16 = QParams(16, 4, -1, False)
    qcfg = [(w4a16, w4a16), (W8A8, W8A8), (w4a16, W8A8), (w4a16, w4a16), (QParams(16, 4, 128, True), w4a16),
            (w4a16, w4a16), (w4a16, w4a16)]
    gu, dn = [w.to(DEV) for w in gate_up], [w.to(DEV) for w in down]
    plain = moe.MoEFFN(gu, dn, qcfg, num_routed=E, fuse_silu=False)
    fused = moe.MoEFFN(gu, dn, qcfg, num_routed=E)
    assert fused.fuse_silu
    logits = torch.rand(T, E, generator=g)
    ids = torch.topk(logits, topk, dim=1).indices.to(torch.int32).to(DEV)
    wts = torch.softmax(torch.rand(T, topk, generator=g), dim=1).to(DEV)
    h = ((torch.rand(T, H, generator=g) * 2 - 1) * 3).half().to(DEV)
    o1, m1 = plain.forward(h, ids, wts, return_intermediates=True)
    o2, m2 = fused.forward(h, ids, wts, return_intermediates=True)
    torch.cuda.synchronize()
    assert torch.equal(m1["a2"].out, m2["a2"].out)
    assert torch.equal(o1.view(torch.int16), o2.view(torch.int16))
    assert moe.PlannedForward(fused, h, ids, wts).mode == mode

