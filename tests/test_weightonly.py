"""Weight-only WxA16 host side (CPU): the reference-format repack, the quantisation restatements,
validation of weight-only problems, and the variant table."""
from __future__ import annotations

import ctypes

import numpy as np
import pytest
import torch

from mxmoe_amd import _native as nat
from mxmoe_amd.quantize import pack_weightonly_mi355x, quant_weightonly
from oracle import weightonly as wo


@pytest.mark.parametrize("bits", [2, 4, 8])
@pytest.mark.parametrize("sym", [True, False])
@pytest.mark.parametrize("N,K", [(64, 128), (256, 1408), (96, 64)])
def test_repack_inverts_reference_packing(bits, sym, N, K):
    if N % (8 * 16 // bits):
        pytest.skip("reference permute_weight needs N % (8 * pack) == 0")
    rng = np.random.default_rng(N * K + bits)
    lo, hi = wo.qrange(bits, sym)
    q = rng.integers(lo, hi + 1, size=(N, K)).astype(np.int32)
    ref = wo.ref_pack(q, bits, sym)
    assert ref.shape == (N * bits // 16, K)
    assert np.array_equal(nat.repack_weightonly(ref, N, K, bits), wo.mi355x_pack(q, bits, sym))


def test_reference_permutation_is_a_bijection():
    for bits in (2, 4, 8):
        perm = wo._perm_indices(bits)
        assert sorted(perm.tolist()) == list(range(len(perm)))


@pytest.mark.parametrize("args,status", [
    ((64, 128, 3), nat.MXMOE_GG_ERR_UNSUPPORTED),
    ((32, 128, 2), nat.MXMOE_GG_ERR_INVALID),  # 2-bit: N % 64
    ((60, 128, 4), nat.MXMOE_GG_ERR_INVALID),
    ((64, 96, 4), nat.MXMOE_GG_ERR_INVALID),
])
def test_repack_rejects_bad_shapes(args, status):
    N, K, bits = args
    src = np.zeros((max(1, N * 8 // 16), K), dtype=np.uint16)
    out = np.zeros((N, K), dtype=np.uint8)
    assert nat.lib().mxmoe_gg_repack_weightonly(src.ctypes.data, N, K, bits, out.ctypes.data) == status


@pytest.mark.parametrize("bits", [2, 4, 8])
@pytest.mark.parametrize("gsize", [-1, 128])
@pytest.mark.parametrize("sym", [True, False])
def test_torch_quantisation_matches_oracle(bits, gsize, sym):
    b = (torch.rand(64, 256, generator=torch.Generator().manual_seed(bits + gsize)) * 2 - 1).to(torch.float16)
    codes, sz = quant_weightonly(b, bits, gsize, sym)
    q, sz_ref = wo.quant_wo(b.numpy(), bits, gsize, sym)
    assert np.array_equal(codes.numpy().astype(np.int32), wo.stored_codes(q, bits, sym))
    assert np.array_equal(sz.numpy().view(np.uint16), wo.permute_scale(sz_ref, 64, 256, gsize, sym).view(np.uint16))
    assert np.array_equal(pack_weightonly_mi355x(codes, bits).numpy(), wo.mi355x_pack(q, bits, sym))
    # the dequantised weights reconstruct the input within half a quantisation step of their group
    deq = wo.dequant(q, wo.permute_scale(sz_ref, 64, 256, gsize, sym), 64, 256, bits, gsize, sym).astype(np.float32)
    g = 256 if gsize == -1 else gsize
    scale = (sz_ref if sym else sz_ref[:, 0]).astype(np.float32).reshape(64, 256 // g)
    bound = np.repeat(scale, g, axis=1) * 0.51 + 2e-3
    assert (np.abs(deq - b.numpy().astype(np.float32)) <= bound).all()


def _prob(**kw):
    d = dict(A=16, B=16, scale_a=0, scale_b=16, C=16, M=64, N=128, K=256, a_bits=16, w_bits=4, gsize=128, sym=0)
    d.update(kw)
    return nat.GGProblemC(**d)


def _plan(problems, variant):
    arr = (nat.GGProblemC * len(problems))(*problems)
    info = nat.GGPlanInfo()
    st = nat.lib().mxmoe_gg_plan(arr, len(problems), variant, None, 0, None, ctypes.byref(info))
    return st, nat.lib().mxmoe_gg_last_error().decode()


def _variant(name):
    return [ln.split()[1] for ln in nat.list_variants()].index(name)


@pytest.mark.parametrize("kw,status,msg", [
    (dict(K=224), nat.MXMOE_GG_ERR_INVALID, "K % 64"),
    (dict(gsize=96, K=384), nat.MXMOE_GG_ERR_UNSUPPORTED, "group size"),
    (dict(gsize=128, K=192), nat.MXMOE_GG_ERR_UNSUPPORTED, "group size"),
    (dict(scale_b=0), nat.MXMOE_GG_ERR_INVALID, "NULL scale"),
    (dict(scale_b=18), nat.MXMOE_GG_ERR_INVALID, "4-byte aligned"),
    (dict(w_bits=3), nat.MXMOE_GG_ERR_UNSUPPORTED, "quant type not supported"),
])
def test_weightonly_validation(kw, status, msg):
    st, err = _plan([_prob(), _prob(**kw)], nat.default_variant())
    assert st == status and msg in err and "problem 1" in err


def test_weightonly_only_on_v2_variants():
    for ln in nat.list_variants():
        vid, name = int(ln.split()[0]), ln.split()[1]
        st, err = _plan([_prob()], vid)
        if name.startswith(("v2", "abl_v2")):
            assert st == nat.MXMOE_GG_ERR_WORKSPACE, (name, err)  # validation passed, no workspace given
            assert "w4a16=TileConfig(BM=256, BN=256, BK=64" in ln and "w8a16=TileConfig(" in ln
        elif name.startswith("wo3"):  # weight-only-only kernel: 64-row tiles, no fp16 / int bodies
            assert st == nat.MXMOE_GG_ERR_WORKSPACE, (name, err)
            assert "w4a16=TileConfig(BM=64, BN=256, BK=64" in ln and "w4a4_g128_sym=" not in ln
            assert "w8a8_g-1_sym=TileConfig(BM=64, BN=128" in ln  # int8 problems may ride along
        else:
            assert st == nat.MXMOE_GG_ERR_UNSUPPORTED and "does not implement" in err, name
            assert "w4a16" not in ln
    # AUTO never routes weight-only problems to a variant without the kernel
    arr = (nat.GGProblemC * 2)(_prob(), _prob(a_bits=4, w_bits=4, gsize=-1, sym=1, scale_a=16))
    assert nat.workspace_size(arr, 2, nat.VARIANT_AUTO) == nat.workspace_size(arr, 2, nat.default_variant())
