"""w4a4 on fp6 images (MXMOE_GG_FMT_F6, mxmoe_amd/csrc/gg_f6.h) — a lab-library route (measured
9-18 % slower than the product's int4 tiles on the layer calls), kept tested
because its exactness argument (int4 codes as FP6 E3M2, f32 sums of small integers) is reusable.
These tests load libmxmoe_gg_lab.so (`python -m mxmoe_amd.build --lab`) in place of the product
library for this module and skip when it is not built.

CPU: the library's image builder (mxmoe_gg_pack_f6_host) against a numpy restatement of the image
layout documented in gg_f6.h, every code decoding (OCP FP6 E3M2) to its int4 value, the
planner's handling of fp6 problems. GPU: the device builder equals the host one byte for byte, and the
GroupGEMM over images equals the w4a4 oracle (oracle.gg_quant on the packed int4 operands) bit for
bit — the same bar as the int4 path — on edge shapes, K tails, empty problems and a full-size layer.
"""
from __future__ import annotations

import ctypes

import numpy as np
import pytest
import torch

from mxmoe_amd import _native as nat
from mxmoe_amd.groupgemm import W4A4, W4A4_F6, W8A8, GroupGemm, Problem, QParams
from oracle import oracle

LAB = nat.LIB_PATH.with_name("libmxmoe_gg_lab.so")


@pytest.fixture(scope="module", autouse=True)
def _lab_lib():
    from mxmoe_amd import build

    if not LAB.exists():
        pytest.skip("lab library not built (python -m mxmoe_amd.build --lab)")
    if build.needs_build(build.LAB_LIB):  # never test a lab binary HEAD does not produce
        pytest.skip("lab library older than its sources (rebuild: python -m mxmoe_amd.build --lab)")
    lab = ctypes.CDLL(str(LAB))
    if not hasattr(lab, "mxmoe_gg_pack_f6"):
        pytest.skip("lab library predates the fp6 route")
    nat._declare(lab)
    saved = nat.lib()
    nat._lib = lab
    yield
    nat._lib = saved


def _np_image(codes: np.ndarray, K: int) -> np.ndarray:
    """numpy restatement of the fp6 image (gg_f6.h header comment, mxmoe_gg_pack_f6)."""
    rows = codes.shape[0]
    nib = np.zeros((rows, (K + 127) // 128 * 128), dtype=np.int64)
    b = codes[:, : K // 2].astype(np.int64)
    nib[:, 0:K:2] = b & 15
    nib[:, 1:K:2] = b >> 4
    val = np.where(nib >= 8, nib - 16, nib)  # two's complement int4
    mag = np.array([0, 12, 16, 18, 20, 21, 22, 23, 24], dtype=np.int64)  # e3m2 codes of 0..8
    code = np.where(val < 0, 32, 0) + mag[np.abs(val)]
    nblk = nib.shape[1] // 128
    out = np.zeros((rows, nblk * 96), dtype=np.uint8)
    for blk in range(nblk):
        for g in range(4):
            c = code[:, blk * 128 + g * 32: blk * 128 + g * 32 + 32]
            big = np.zeros(rows, dtype=object)
            for j in range(32):
                big = big + (c[:, j].astype(object) << (6 * j))
            for d in range(6):
                w = np.array([(int(x) >> (32 * d)) & 0xFFFFFFFF for x in big], dtype=np.uint32)
                off = blk * 96 + (g * 16 + 4 * d if d < 4 else 64 + g * 8 + 4 * (d - 4))
                out[:, off: off + 4] = w.view(np.uint8).reshape(rows, 4)
    return out


def _decode_e3m2(c: np.ndarray) -> np.ndarray:
    sign = np.where(c & 32, -1.0, 1.0)
    e, m = (c >> 2) & 7, c & 3
    v = np.where(e == 0, m / 4.0 * 2.0 ** -2, (1 + m / 4.0) * 2.0 ** (e.astype(np.float64) - 3))
    return sign * v


def _image_values(img: np.ndarray, K: int) -> np.ndarray:
    """Decode an image back to the element values in image order (element e = nibble e)."""
    rows = img.shape[0]
    nblk = img.shape[1] // 96
    out = np.zeros((rows, nblk * 128))
    for blk in range(nblk):
        for g in range(4):
            base = blk * 96
            dw = np.concatenate([img[:, base + g * 16: base + g * 16 + 16], img[:, base + 64 + g * 8: base + 72 + g * 8]],
                                axis=1).view(np.uint32)
            for j in range(32):
                bit = 6 * j
                lo = dw[:, bit // 32].astype(np.uint64) >> np.uint64(bit % 32)
                if bit % 32 > 26:
                    lo |= dw[:, bit // 32 + 1].astype(np.uint64) << np.uint64(32 - bit % 32)
                out[:, blk * 128 + g * 32 + j] = _decode_e3m2((lo & np.uint64(63)).astype(np.int64))
    return out[:, :K], out[:, K:]


@pytest.mark.parametrize("K", [32, 96, 128, 160, 1408, 2048])
def test_host_image_matches_numpy_restatement(K):
    rng = np.random.default_rng(K)
    codes = rng.integers(0, 256, size=(5, K // 2), dtype=np.uint8)
    got = nat.pack_f6_host(codes, K)
    assert got.shape == (5, nat.f6_row_bytes(K))
    assert (got == _np_image(codes, K)).all()


def test_image_decodes_to_the_int4_values_and_zero_padding():
    K = 160  # one full K-128 block + a 32-element tail block
    codes = np.arange(256, dtype=np.uint8)[None, :].repeat(2, 0)[:, : K // 2]
    img = nat.pack_f6_host(codes, K)
    vals, pad = _image_values(img, K)
    nib = np.zeros((2, K), dtype=np.int64)
    nib[:, 0::2], nib[:, 1::2] = codes & 15, codes >> 4
    assert (vals == np.where(nib >= 8, nib - 16, nib)).all()  # every int4 value -8..7 exact
    assert (pad == 0).all()


def test_image_dot_products_are_the_int4_dot_products():
    # the kernel's claim: the sum over image elements equals the packed-int4 dot product, exactly
    K = 384
    rng = np.random.default_rng(1)
    a4 = rng.integers(0, 256, size=(7, K // 2), dtype=np.uint8)
    b4 = rng.integers(0, 256, size=(9, K // 2), dtype=np.uint8)
    va, _ = _image_values(nat.pack_f6_host(a4, K), K)
    vb, _ = _image_values(nat.pack_f6_host(b4, K), K)
    qa = oracle.unpack_wxax(a4, 4, K).astype(np.int64)
    qb = oracle.unpack_wxax(b4, 4, K).astype(np.int64)
    assert (va @ vb.T == (qa @ qb.T).astype(np.float64)).all()


def test_pack_rejects_bad_arguments():
    with pytest.raises(nat.GGError):
        nat.pack_f6_host(np.zeros((2, 24), dtype=np.uint8), 48)  # K % 32 != 0


def _cproblems(specs):
    ps = []
    for M, N, K, q in specs:
        ps.append(nat.GGProblemC(A=16, B=16, scale_a=16, scale_b=16, C=16, M=M, N=N, K=K, a_bits=q.a_bits,
                                 w_bits=q.w_bits, gsize=q.gsize, sym=int(q.sym), fmt=q.fmt_code, lda=0, ldb=0, ldc=0))
    return (nat.GGProblemC * len(ps))(*ps)


def test_auto_picks_the_fp6_kernel_and_rejects_mixing():
    arr = _cproblems([(300, 256, 2048, W4A4_F6), (129, 512, 1408, W4A4_F6), (0, 256, 256, W4A4_F6)])
    v = nat.resolve_variant(arr, 3)
    assert nat.list_variants()[v].split()[1] == "f6_256x256_w8_ring3"
    tiles, rows = nat.plan_tiles(list(arr), v)
    live = tiles[tiles[:, 0] >= 0]
    # 300 rows: one 256-row tile + one 128-row tail tile per n-tile; 129 rows: 256-row class
    assert sorted(set(live[:, 3] & 0xFF)) == [0, 1]
    assert len(live) == 2 * 1 + 1 * 2
    with pytest.raises(nat.GGError, match="cannot share a call"):
        nat.resolve_variant(_cproblems([(300, 256, 2048, W4A4_F6), (64, 256, 256, W8A8)]), 2)
    # no other variant reads fp6 images
    d = nat.default_variant()
    with pytest.raises(nat.GGError):
        nat.workspace_size(_cproblems([(64, 256, 256, W4A4_F6)]), 1, d)


def test_qcfg_round_trip():
    assert W4A4_F6.qcfg == "w4a4_g-1_sym_F6"
    assert QParams.from_qcfg("w4a4_g-1_sym_F6") == W4A4_F6


# ---------------------------------------------------------------- GPU
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


class _F6Problem:
    def __init__(self, M, N, K, seed):
        from mxmoe_amd.quantize import pack_wxax, quant_rtn_sym

        g = torch.Generator().manual_seed(seed)
        a = (torch.rand(M, K, generator=g) * 2 - 1).to(torch.float16)
        b = (torch.rand(N, K, generator=g) * 2 - 1).to(torch.float16)
        qa, sa = quant_rtn_sym(a, 4, -1)
        qb, sb = quant_rtn_sym(b, 4, -1)
        self.M, self.N, self.K = M, N, K
        self.A4, self.B4 = pack_wxax(qa, 4).numpy(), pack_wxax(qb, 4).numpy()
        self.sa, self.sb = sa.numpy(), sb.numpy()
        dev = torch.device("cuda")
        self.C = torch.full((max(M, 1), N), float("nan"), dtype=torch.float16, device=dev)
        A = nat.pack_f6(torch.from_numpy(self.A4).to(dev), K)
        B = nat.pack_f6(torch.from_numpy(self.B4).to(dev), K)
        self.problem = Problem(A=A, B=B, C=self.C, M=M, N=N, K=K, q=W4A4_F6, scale_a=torch.from_numpy(self.sa).to(dev),
                               scale_b=torch.from_numpy(self.sb).to(dev))

    def check(self):
        out = self.C[: self.M].cpu().numpy()
        ref = oracle.gg_quant(self.A4, self.B4, self.sa, self.sb, self.M, self.N, self.K, 4)
        mism = np.count_nonzero(out.view(np.uint16) != ref.view(np.uint16))
        assert mism == 0, f"fp6 w4a4 M={self.M} N={self.N} K={self.K}: {mism} mismatching outputs"


@pytest.mark.gpu
@pytest.mark.parametrize("K", [32, 96, 128, 160, 1408, 2048])
def test_device_image_equals_host_image(K):
    _gpu()
    rng = np.random.default_rng(K)
    codes = rng.integers(0, 256, size=(37, K // 2), dtype=np.uint8)
    dev = nat.pack_f6(torch.from_numpy(codes).cuda(), K)
    torch.cuda.synchronize()
    assert (dev.cpu().numpy() == nat.pack_f6_host(codes, K)).all()
    # strided source and destination rows
    src = torch.zeros((37, K // 2 + 16), dtype=torch.uint8, device="cuda")
    src[:, : K // 2] = torch.from_numpy(codes).cuda()
    dst = torch.zeros((37, nat.f6_row_bytes(K) + 32), dtype=torch.uint8, device="cuda")
    nat.pack_f6(src[:, : K // 2], K, out=dst[:, : nat.f6_row_bytes(K)])
    torch.cuda.synchronize()
    assert (dst[:, : nat.f6_row_bytes(K)].cpu().numpy() == nat.pack_f6_host(codes, K)).all()
    assert (dst[:, nat.f6_row_bytes(K):] == 0).all()


@pytest.mark.gpu
def test_fp6_gemm_edge_shapes_bit_exact():
    _gpu()
    shapes = [(1, 128, 256), (17, 256, 128), (130, 128, 384), (257, 136, 512), (64, 8, 1024), (300, 520, 512),
              (513, 264, 256), (0, 256, 256), (129, 384, 160), (77, 128, 96), (384, 512, 1408), (5, 128, 32)]
    hps = [_F6Problem(M, N, K, seed=200 + i) for i, (M, N, K) in enumerate(shapes)]
    gg = GroupGemm([h.problem for h in hps])
    assert nat.list_variants()[gg.variant].split()[1] == "f6_256x256_w8_ring3"
    gg.launch()
    torch.cuda.synchronize()
    for h in hps:
        h.check()
    gg.launch()  # relaunch on the same plan: identical
    torch.cuda.synchronize()
    for h in hps:
        h.check()


@pytest.mark.gpu
def test_fp6_gemm_extreme_codes_long_k():
    # all codes -8 (the largest products) at K = 14336: partial sums up to 917504, exact in f32
    _gpu()
    M, N, K = 300, 256, 14336
    dev = torch.device("cuda")
    A4 = torch.full((M, K // 2), 0x88, dtype=torch.uint8, device=dev)
    B4 = torch.full((N, K // 2), 0x88, dtype=torch.uint8, device=dev)
    B4[1::2] = 0x77  # +7 columns too
    sa = torch.full((M,), 2.0 ** -10, dtype=torch.float16, device=dev)
    sb = torch.full((N,), 2.0 ** -10, dtype=torch.float16, device=dev)
    C = torch.empty((M, N), dtype=torch.float16, device=dev)
    p = Problem(A=nat.pack_f6(A4, K), B=nat.pack_f6(B4, K), C=C, M=M, N=N, K=K, q=W4A4_F6, scale_a=sa, scale_b=sb)
    GroupGemm([p]).launch()
    torch.cuda.synchronize()
    ref = oracle.gg_quant(A4.cpu().numpy(), B4.cpu().numpy(), sa.cpu().numpy(), sb.cpu().numpy(), M, N, K, 4)
    assert (C.cpu().numpy().view(np.uint16) == ref.view(np.uint16)).all()


@pytest.mark.gpu
def test_fp6_equals_int4_path_full_size_w4a4_layer():
    """BASELINE configs[2]-shape w4a4 layer (qwen2_moe layer 11, bs 8192): the fp6-image call returns
    the int4 call's outputs bit for bit (every problem, every element), and sampled rows match the
    oracle."""
    _gpu()
    from mxmoe_amd.harness import F6Layer, build_layer_inputs
    from tests._util import full_size_layer

    wl = full_size_layer("w4a4")
    for gg in ("gate_up", "down"):
        inp = build_layer_inputs(wl[gg])
        GroupGemm(inp.problems).launch()
        torch.cuda.synchronize()
        ref = [p.C.clone() for p in inp.problems]
        f6 = F6Layer(inp)
        for p in f6.problems:
            p.C.fill_(float("nan"))
        g6 = GroupGemm(f6.problems)
        f6.pack_a()
        g6.launch()
        torch.cuda.synchronize()
        for r, p in zip(ref, f6.problems):
            assert torch.equal(r[: p.M].view(torch.int16), p.C[: p.M].view(torch.int16)), f"M={p.M} N={p.N} K={p.K}"
        del inp, f6, g6, ref
        torch.cuda.empty_cache()
