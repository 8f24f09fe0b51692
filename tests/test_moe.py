"""MoE-layer plumbing: routing, activation quantisation, SiLU·mul + quant,
combine, and the MoEFFN layer built from them and the fused GroupGEMM.

Reference: ref_bind.cu (gg_permute_inp :47-64, quant_inp_act :434-592, silu_mul_then_quant :595-757,
gg_unpermute_out :66). The reference's device kernels (act_kernel.cuh) are absent, so the oracle
(oracle/moe_ref.py) restates the reference's quant_weight + pack_wxax per token row; routing and
quantisation are bit-exact, the SiLU (expf: libm vs ocml) is held to 1 fp16 ulp / 1 code step.
"""
from __future__ import annotations

import ctypes

import numpy as np
import pytest
import torch

from mxmoe_amd import _native as nat
from mxmoe_amd import moe
from mxmoe_amd.groupgemm import FP16, W4A4, W4A4_G128, W8A8, QParams
from oracle import moe_ref, oracle

DEV = "cuda"


def _ids(T, topk, E, seed):
    g = torch.Generator().manual_seed(seed)
    # distinct experts per token, skewed popularity, one expert left empty
    logits = torch.rand(T, E, generator=g) + torch.linspace(0, 1.5, E)
    logits[:, 3] = -1.0
    return torch.topk(logits, topk, dim=1).indices.to(torch.int32)


# ------------------------------------------------------------------------------------------ CPU

def test_oracle_route_equals_stable_torch_sort():
    ids = _ids(50, 4, 8, 0)
    sorted_e, perm, inv, counts = moe_ref.route(ids.numpy(), 8)
    v, idx = torch.sort(ids.view(-1).to(torch.int64), stable=True)
    assert (sorted_e == v.numpy()).all()
    assert (perm == (idx // 4).numpy()).all()
    assert (counts == torch.bincount(ids.view(-1).to(torch.int64), minlength=8).numpy()).all()
    assert (sorted_e[inv] == ids.view(-1).numpy()).all()


def test_qtag_mapping_follows_reference():
    assert moe.qtag_of(16, -1) == moe.ACT_FP16
    assert moe.qtag_of(8, -1) == moe.ACT_INT8
    assert moe.qtag_of(4, -1) == moe.ACT_INT4
    assert moe.qtag_of(4, 128) == moe.ACT_INT4_G128
    with pytest.raises(ValueError):
        moe.qtag_of(8, 128)


def test_abi_validation_without_gpu():
    lib = nat.lib()
    assert lib.mxmoe_moe_quant_act(None, 4, 100, 2, 0, None, None, None, 1, None, None, None) == nat.MXMOE_GG_ERR_INVALID
    assert b"K % 128" in lib.mxmoe_gg_last_error()
    assert lib.mxmoe_moe_combine(None, None, None, None, None, 4, 2, 12, None, None) == nat.MXMOE_GG_ERR_INVALID
    assert lib.mxmoe_moe_route(None, 4, 2, 0, None, None, None, None, None) == nat.MXMOE_GG_ERR_INVALID
    # the fused-SiLU companions (round 5): widths must be multiples of 128, pointers 16-B aligned
    for fn in (lib.mxmoe_moe_quant_slots, lib.mxmoe_moe_silu_mul_quant_il, lib.mxmoe_moe_silu_mul_quant):
        assert fn(None, None, 4, 2, 100, 0, None, None, 1, None, None, None) == nat.MXMOE_GG_ERR_INVALID
        assert b"multiples of 128" in lib.mxmoe_gg_last_error()
        assert fn(None, None, 4, 2, 128, 0, None, None, 1, None, None, None) == nat.MXMOE_GG_ERR_INVALID
        assert b"NULL or misaligned" in lib.mxmoe_gg_last_error()
        assert fn(None, None, 0, 2, 128, 0, None, None, 1, None, None, None) == nat.MXMOE_GG_OK  # T = 0: nothing
    assert ctypes.sizeof(nat.MoeSegC) == 32


# ------------------------------------------------------------------------------------------ GPU

@pytest.fixture()
def gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    nat.lib()


def _hidden(T, K, seed):
    g = torch.Generator().manual_seed(seed)
    return ((torch.rand(T, K, generator=g) * 2 - 1) * 3).half()


@pytest.mark.gpu
@pytest.mark.parametrize("T,topk,E", [(1, 1, 4), (50, 4, 8), (1000, 6, 64), (4096, 4, 60)])
def test_route_matches_oracle(gpu, T, topk, E):
    ids = _ids(T, topk, E, T)
    r = moe.route(ids.to(DEV), E)
    torch.cuda.synchronize()
    sorted_e, perm, inv, counts = moe_ref.route(ids.numpy(), E)
    assert r.counts == counts.tolist()
    assert (r.sorted_expert.cpu().numpy() == sorted_e).all()
    assert (r.perm_token.cpu().numpy() == perm).all()
    assert (r.inv_slot.cpu().numpy() == inv).all()


def _check_batch(b, expect_rows, tags):
    for e, (rows, tag) in enumerate(zip(expect_rows, tags)):
        if rows.shape[0] == 0:
            continue
        stored, scale = moe_ref.quant_rows(rows, tag)
        got = b.A(e).cpu().numpy()
        if tag == moe.ACT_FP16:
            assert (got.view(np.uint16) == stored.view(np.uint16)).all(), f"seg {e}"
        else:
            assert (got == stored).all(), f"seg {e} tag {tag}"
            assert (b.scale(e).cpu().numpy().view(np.uint16) == scale.view(np.uint16)).all(), f"seg {e} scales"


@pytest.mark.gpu
@pytest.mark.parametrize("K", [256, 2048, 5632])
# (33, 3): an odd number of routed slots, so the last wave of the two-rows-per-wave launch holds one row
@pytest.mark.parametrize("T,topk", [(97, 4), (33, 3)])
def test_quant_act_bit_exact(gpu, K, T, topk):
    E = 8
    ids = _ids(T, topk, E, 1)
    h = _hidden(T, K, 2)
    tags = [0, 1, 2, 3, 1, 2, 0, 3, 1]  # shared expert last (int8)
    r = moe.route(ids.to(DEV), E)
    b = moe.quant_act(h.to(DEV), r, tags, with_shared=True)
    torch.cuda.synchronize()
    sorted_e, perm, inv, counts = moe_ref.route(ids.numpy(), E)
    gathered = h.numpy()[perm]
    starts = np.concatenate([[0], np.cumsum(counts)])
    rows = [gathered[starts[e]:starts[e + 1]] for e in range(E)] + [h.numpy()]
    _check_batch(b, rows, tags)


@pytest.mark.gpu
def test_gg_permute_inp_mirror(gpu):
    T, topk, E, K = 33, 2, 6, 384
    ids = _ids(T, topk, E, 5)
    h = _hidden(T, K, 6).to(DEV)
    n, inp, idx, cnt = moe.gg_permute_inp(h, ids.to(DEV), E)
    v, order = torch.sort(ids.view(-1).to(torch.int64), stable=True)
    ref = h.index_select(0, (order // topk).to(DEV))
    assert torch.equal(inp.view(torch.int16), ref.view(torch.int16))
    assert n == int((cnt > 0).sum())


@pytest.mark.gpu
# (256, 640): the shared row's quarter runs are 256, 256, 128 and 0 columns (one launch, split rows)
@pytest.mark.parametrize("N,Ns", [(256, 512), (1408, 5632), (256, 640), (512, 512)])
@pytest.mark.parametrize("shared_tag", [0, 1, 2, 3])
@pytest.mark.parametrize("T,topk", [(61, 4), (33, 3)])
def test_silu_mul_quant_within_one_step(gpu, N, Ns, shared_tag, T, topk):
    E = 8
    ids = _ids(T, topk, E, 7)
    r = moe.route(ids.to(DEV), E)
    g = torch.Generator().manual_seed(8)
    routed = ((torch.rand(T * topk, 2 * N, generator=g) * 2 - 1) * 4).half()
    shared = ((torch.rand(T, 2 * Ns, generator=g) * 2 - 1) * 4).half()
    tags = [0, 1, 2, 3, 0, 1, 2, 3, shared_tag]
    b = moe.silu_mul_quant(routed.to(DEV), shared.to(DEV), r, tags)
    torch.cuda.synchronize()
    act_r = moe_ref.silu_mul(routed.numpy())
    act_s = moe_ref.silu_mul(shared.numpy())
    starts = np.concatenate([[0], np.cumsum(r.counts)])
    rows = [act_r[starts[e]:starts[e + 1]] for e in range(E)] + [act_s]
    exact = total = 0
    for e, (x, tag) in enumerate(zip(rows, tags)):
        if x.shape[0] == 0:
            continue
        got = b.A(e).cpu().numpy()
        if tag == moe.ACT_FP16:  # the act itself: within 1 fp16 ulp of the libm restatement
            d = np.abs(got.view(np.int16).astype(np.int32) - x.view(np.int16).astype(np.int32))
            assert d.max() <= 1, f"seg {e}: act differs by {d.max()} ulp"
            exact += int((d == 0).sum())
            total += d.size
            continue
        bits = 8 if tag == moe.ACT_INT8 else 4
        W = x.shape[1]
        qg = oracle.unpack_wxax(got, bits, W).astype(np.int32)
        stored, sc = moe_ref.quant_rows(x, tag)
        qr = oracle.unpack_wxax(stored, bits, W).astype(np.int32)
        sg = b.scale(e).cpu().numpy()
        ds = np.abs(sg.view(np.int16).astype(np.int32) - sc.view(np.int16).astype(np.int32))
        assert ds.max() <= 1, f"seg {e}: scales differ by {ds.max()} ulp"
        assert np.abs(qg - qr).max() <= 1, f"seg {e}: codes differ by more than one step"
        exact += int((qg == qr).sum())
        total += qg.size
    assert exact / total > 0.995, f"only {exact}/{total} exact"


@pytest.mark.gpu
@pytest.mark.parametrize("shared", [False, True])
def test_combine_bit_exact(gpu, shared):
    T, topk, E, H = 77, 4, 8, 2048
    ids = _ids(T, topk, E, 9)
    r = moe.route(ids.to(DEV), E)
    g = torch.Generator().manual_seed(10)
    y = ((torch.rand(T * topk, H, generator=g) * 2 - 1)).half()
    w = torch.softmax(torch.rand(T, topk, generator=g), dim=1)
    sh = (torch.rand(T, H, generator=g) * 2 - 1).half() if shared else None
    sw = torch.rand(T, generator=g) if shared else None
    out = moe.combine(y.to(DEV), r, w.to(DEV), None if sh is None else sh.to(DEV), None if sw is None else sw.to(DEV))
    torch.cuda.synchronize()
    ref = moe_ref.combine(y.numpy(), r.inv_slot.cpu().numpy(), w.numpy(), topk,
                          None if sh is None else sh.numpy(), None if sw is None else sw.numpy())
    assert (out.cpu().numpy().view(np.uint16) == ref.view(np.uint16)).all()


@pytest.mark.gpu
def test_moe_ffn_stagewise_parity(gpu):
    """Every stage of MoEFFN.forward checked against the oracle given the previous stage's GPU output
    (routing / quant / GroupGEMM / combine bit-exact; the fused SiLU within one code step)."""
    T, topk, E, H, N, Ns = 120, 4, 6, 256, 256, 512
    g = torch.Generator().manual_seed(11)
    gate_up = [((torch.rand(2 * N, H, generator=g) * 2 - 1) * 0.2).half() for _ in range(E)]
    gate_up.append(((torch.rand(2 * Ns, H, generator=g) * 2 - 1) * 0.2).half())
    down = [((torch.rand(H, N, generator=g) * 2 - 1) * 0.2).half() for _ in range(E)]
    down.append(((torch.rand(H, Ns, generator=g) * 2 - 1) * 0.2).half())
    qcfg = [(W8A8, W8A8), (W4A4, W8A8), (W4A4_G128, W4A4_G128), (FP16, FP16), (W8A8, W4A4),
            (QParams(16, 4, 128, False), FP16), (W8A8, W4A4_G128)]
    layer = moe.MoEFFN([w.to(DEV) for w in gate_up], [w.to(DEV) for w in down], qcfg, num_routed=E)
    ids = _ids(T, topk, E, 12)
    wts = torch.softmax(torch.rand(T, topk, generator=g), dim=1)
    h = _hidden(T, H, 13)
    out, mid = layer.forward(h.to(DEV), ids.to(DEV), wts.to(DEV), return_intermediates=True)
    torch.cuda.synchronize()
    r, a1, h1, h1s, a2, y, ys = (mid[k] for k in ("routing", "a1", "h1", "h1s", "a2", "y", "ys"))
    # gate_up GroupGEMM outputs from the GPU's own quantised activations (bit-exact int paths)
    for e, s in enumerate(a1.segs):
        if s.rows == 0:
            continue
        w = layer.w1[e]
        C = (h1s if e == E else h1[s.first_slot:s.first_slot + s.rows]).cpu().numpy()
        A = a1.A(e).cpu().numpy()
        if w.q.is_weight_only:
            from oracle import weightonly  # noqa: F401 — weight-only: tolerance-checked in its own tests
            continue
        if not w.q.is_quant:
            ref = oracle.gg_f16(A, w.B.cpu().numpy(), s.rows, w.N, w.K)
            err = np.abs(C.astype(np.float64) - ref.astype(np.float64))
            assert (err <= 1e-3 * np.abs(ref) + 1e-3 * np.sqrt(np.mean(ref.astype(np.float64) ** 2)) + 1e-6).all()
            continue
        sa, sb = a1.scale(e).cpu().numpy(), w.scale_b.cpu().numpy()
        if w.q.gsize == 128:
            ref = oracle.gg_quant_grouped(A, w.B.cpu().numpy(), sa, sb, s.rows, w.N, w.K, 4, 128)
        else:
            ref = oracle.gg_quant(A, w.B.cpu().numpy(), sa, sb, s.rows, w.N, w.K, w.q.a_bits)
        assert (C.view(np.uint16) == ref.view(np.uint16)).all(), f"gate_up expert {e}"
    # combine of the GPU's down outputs
    ref = moe_ref.combine(y.cpu().numpy(), r.inv_slot.cpu().numpy(), wts.numpy(), topk, ys.cpu().numpy())
    assert (out.cpu().numpy().view(np.uint16) == ref.view(np.uint16)).all()
    assert torch.isfinite(out.float()).all()


@pytest.mark.gpu
def test_gg_mxmoe_share_fused_mirror(gpu):
    """The reference-named fused GroupGEMM op (ref_bind.cu:312-431) on quant_inp_act's outputs:
    per-problem inputs / scales / outputs, per-expert weights / qparams, the shared expert last.
    Bit-exact against the oracle for every integer problem; a second call with new activations on
    the same routing reuses the cached plan (mxmoe_gg_rebind) and is exact again."""
    T, topk, E, H, N = 90, 4, 6, 256, 256
    g = torch.Generator().manual_seed(21)
    qs = [W8A8, W4A4, W8A8, W4A4, W8A8, W4A4, W8A8]  # shared expert last
    qparams = [(q.a_bits, q.w_bits, q.gsize, q.sym) for q in qs]
    ws = [moe.prepare_weight((((torch.rand(2 * N, H, generator=g) * 2 - 1) * 0.2).half()).to(DEV), q) for q in qs]
    ids = _ids(T, topk, E, 22)
    for call, seed in enumerate((23, 24)):
        h = _hidden(T, H, seed).to(DEV)
        inp, sc, out, *_rest = moe.quant_inp_act(h, ids.to(DEV), E, N, 1, qparams)
        counts = _rest[3]
        res = moe.gg_mxmoe_share_fused(inp, [w.B for w in ws], sc, [w.scale_b for w in ws], out, 2 * N, H, 2 * N, H,
                                       qparams, counts)
        assert res is out
        torch.cuda.synchronize()
        experts = [e for e in range(E) if int(counts[e]) > 0] + [E]
        assert len(experts) == len(inp)
        for pi, e in enumerate(experts):
            w = ws[e]
            A, sa = inp[pi].cpu().numpy(), sc[pi].cpu().numpy()
            M = A.shape[0]
            ref = oracle.gg_quant(A, w.B.cpu().numpy(), sa, w.scale_b.cpu().numpy(), M, w.N, w.K, w.q.a_bits)
            got = out[pi].cpu().numpy()
            assert (got.view(np.uint16) == ref.view(np.uint16)).all(), f"call {call} expert {e}"
    assert len(moe._SHARE_FUSED_PLANS) >= 1


def test_fast_quotient_matches_ieee_division():
    """moe_ops.hip div_f16_operands: q = x*r, q' = fma(fma(-q, s, x), r, q) with r = rcp(s) within
    1 ulp rounds to the same fp16 as the IEEE f32 quotient for fp16 x and s (the quantiser's
    fp16(x / scale)). Checked here for every positive finite fp16 scale, 64 random x per scale in
    the quantiser's range |x / s| <= 130, and r correctly rounded or 1 ulp off either way; fma is
    emulated exactly in float64 (24-bit x 24-bit products are exact there). Signed zeros may
    differ (-0 vs +0); the integer codes cannot."""
    import warnings

    rng = np.random.default_rng(0)
    s_all = np.arange(1, 0x7C00, dtype=np.uint16).view(np.float16).astype(np.float32)
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        for _ in range(64):
            x = (rng.uniform(-130, 130, size=s_all.shape).astype(np.float32) * s_all).astype(np.float16)
            ok = np.isfinite(x)
            x, s = x[ok].astype(np.float32), s_all[ok]
            ref = np.rint(np.clip((x / s).astype(np.float16).astype(np.float32), -127, 127))
            r0 = (np.float32(1) / s).astype(np.float32)
            for r in (r0, np.nextafter(r0, np.float32(np.inf)), np.nextafter(r0, np.float32(0))):
                q = (x * r).astype(np.float32)
                e = (x.astype(np.float64) - q.astype(np.float64) * s).astype(np.float32)
                q2 = (e.astype(np.float64) * r + q.astype(np.float64)).astype(np.float32)
                got = np.rint(np.clip(q2.astype(np.float16).astype(np.float32), -127, 127))
                assert (got == ref).all()


@pytest.mark.gpu
def test_gg_mxmoe_share_fused_streams_and_strided_output(gpu):
    """The share_fused plan cache keys on the stream and the operand strides: the same
    shapes launched on two streams get two plans (a rebind on one stream never re-points a launch
    in flight on the other), and an output written through a strided view (ldc > N) re-plans instead
    of raising. Both are bit-exact against the oracle."""
    T, topk, E, H, N = 64, 2, 5, 256, 128  # (_ids leaves expert 3 empty)
    g = torch.Generator().manual_seed(31)
    qs = [W8A8, W4A4, W8A8, W4A4, W8A8, W8A8]
    qparams = [(q.a_bits, q.w_bits, q.gsize, q.sym) for q in qs]
    ws = [moe.prepare_weight((((torch.rand(2 * N, H, generator=g) * 2 - 1) * 0.2).half()).to(DEV), q) for q in qs]
    ids = _ids(T, topk, E, 32)
    moe._SHARE_FUSED_PLANS.clear()
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    h = _hidden(T, H, 33).to(DEV)
    inp, sc, out, *_rest = moe.quant_inp_act(h, ids.to(DEV), E, N, 1, qparams)
    counts = _rest[3]
    torch.cuda.synchronize()
    wide = [torch.zeros(o.shape[0], 2 * N + 64, dtype=torch.float16, device=DEV) for o in out]
    outs = {"s1": [torch.empty_like(o) for o in out], "s2": [torch.empty_like(o) for o in out],
            "strided": [w[:, 16:16 + 2 * N] for w in wide]}
    for name, st in (("s1", s1), ("s2", s2), ("strided", s1)):
        moe.gg_mxmoe_share_fused(inp, [w.B for w in ws], sc, [w.scale_b for w in ws], outs[name], 2 * N, H, 2 * N, H,
                                 qparams, counts, stream=st)
    torch.cuda.synchronize()
    assert len(moe._SHARE_FUSED_PLANS) == 3  # s1, s2 and the strided s1 plan
    experts = [e for e in range(E) if int(counts[e]) > 0] + [E]
    for pi, e in enumerate(experts):
        w = ws[e]
        A, sa = inp[pi].cpu().numpy(), sc[pi].cpu().numpy()
        ref = oracle.gg_quant(A, w.B.cpu().numpy(), sa, w.scale_b.cpu().numpy(), A.shape[0], w.N, w.K, w.q.a_bits)
        for name in outs:
            got = outs[name][pi].cpu().numpy()
            assert (got.view(np.uint16) == ref.view(np.uint16)).all(), f"{name} expert {e}"
        assert (wide[pi][:, :16] == 0).all() and (wide[pi][:, 16 + 2 * N:] == 0).all()  # nothing outside the view
