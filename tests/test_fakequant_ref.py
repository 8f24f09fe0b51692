"""Pin the oracle's GroupGEMM OUTPUT (not only its inputs) to code the reference itself executes.

tests/golden/gg_fakequant_ref.npz holds, for every quantised problem of the committed GroupGEMM
vectors, C_fq = F.linear(Quantizer.fake_quant(a), Quantizer.fake_quant(b)) computed by the
reference's own Quantizer (mxmoe/quant/quant.py:87-106, run in the build container by
tests/golden/make_golden.py); and weight-only vectors (w2/w4/w8 a16, g-1 / g128, sym / asym) with
the reference's quant_minmax codes / scales / zero points of B (quant.py:40-84) and
C_fq = F.linear(A, Quantizer(bits, sym, gsize).fake_quant(B)).

CPU side: the C oracle / weight-only restatement agree with C_fq within the stated fake-quant
tolerance (tests/_util.assert_fakequant_close), and the weight-only quantiser reproduces the
reference's asym / sym codes, scales and zero points bit for bit. The HIP side of the same
comparison is tests/test_fakequant_gpu.py.
"""
from __future__ import annotations

from pathlib import Path

import numpy as np
import pytest

from oracle import oracle, weightonly
from tests._util import assert_fakequant_close

GOLD = Path(__file__).resolve().parent / "golden"
FQ = GOLD / "gg_fakequant_ref.npz"
KINDS = {"w8a8": "gg_w8a8_small.npz", "w4a4": "gg_w4a4_small.npz", "mixed": "gg_mixed_small.npz",
         "w4a4g128": "gg_w4a4g128_small.npz"}


def quant_problems(kind):
    """(i, M, N, K, bits, gsize, fixture, C_fq) of every quantised problem of one golden file."""
    fq = np.load(FQ)
    d = np.load(GOLD / KINDS[kind])
    for i in range(int(d["P"])):
        key = f"{kind}_p{i}_Cfq"
        if key not in fq.files:
            continue
        M, N, K = (int(x) for x in d[f"p{i}_shape"])
        yield i, M, N, K, int(d[f"p{i}_bits"]), (128 if kind == "w4a4g128" else -1), d, fq[key]


def wo_problems():
    fq = np.load(FQ)
    for i in range(int(fq["wo_P"])):
        M, N, K, bits, gsize, sym = (int(x) for x in fq[f"wo{i}_spec"])
        yield i, M, N, K, bits, gsize, bool(sym), fq


def test_fixture_covers_every_quant_type():
    seen = {(bits, g) for kind in KINDS for _, _, _, _, bits, g, _, _ in quant_problems(kind)}
    assert seen == {(8, -1), (4, -1), (4, 128)}
    wo = {(bits, g, sym) for _, _, _, _, bits, g, sym, _ in wo_problems()}
    assert {b for b, _, _ in wo} == {2, 4, 8} and {g for _, g, _ in wo} == {-1, 128} and {s for *_, s in wo} == {True, False}


@pytest.mark.parametrize("kind", list(KINDS))
def test_oracle_matches_reference_fake_quant(kind):
    n = 0
    for i, M, N, K, bits, gsize, d, cfq in quant_problems(kind):
        if gsize == -1:
            C = oracle.gg_quant(d[f"p{i}_A"], d[f"p{i}_B"], d[f"p{i}_sa"], d[f"p{i}_sb"], M, N, K, bits)
        else:
            C = oracle.gg_quant_grouped(d[f"p{i}_A"], d[f"p{i}_B"], d[f"p{i}_sa"], d[f"p{i}_sb"], M, N, K, bits, gsize)
        assert (C.view(np.uint16) == d[f"p{i}_C"].view(np.uint16)).all()  # the restatements agree bit for bit
        assert_fakequant_close(C, cfq, f"{kind} p{i}")
        n += M > 0
    assert n >= 4


@pytest.mark.parametrize("i", range(10))
def test_weightonly_quantiser_is_reference_quant_minmax(i):
    """Asym and sym RTN of B (quant_weight restatement) == the reference's quant_minmax, bit for bit."""
    _, M, N, K, bits, gsize, sym, fq = list(wo_problems())[i]
    q, sz = weightonly.quant_wo(fq[f"wo{i}_B"], bits, gsize, sym)
    G = 1 if gsize == -1 else K // gsize
    s = sz.reshape(N, G) if sym else sz.reshape(N, G, 2)[..., 0]
    z = np.zeros_like(s) if sym else sz.reshape(N, G, 2)[..., 1]
    assert (q == fq[f"wo{i}_q"].astype(np.int32)).all()
    assert (s.view(np.uint16) == fq[f"wo{i}_scale"].view(np.uint16)).all()
    assert (z.view(np.uint16) == fq[f"wo{i}_zp"].view(np.uint16)).all()


@pytest.mark.parametrize("i", range(10))
def test_weightonly_oracle_matches_reference_fake_quant(i):
    _, M, N, K, bits, gsize, sym, fq = list(wo_problems())[i]
    q, sz = weightonly.quant_wo(fq[f"wo{i}_B"], bits, gsize, sym)
    sk = weightonly.permute_scale(sz, N, K, gsize, sym)
    C = weightonly.gemm(fq[f"wo{i}_A"], weightonly.dequant(q, sk, N, K, bits, gsize, sym))
    assert_fakequant_close(C, fq[f"wo{i}_Cfq"], f"w{bits}a16 g{gsize} {'sym' if sym else 'asym'}")
