"""C-ABI tests that need no GPU: the library loads, exports exactly what include/*.h declare,
struct layouts match the reference's, and host-side validation rejects bad problems with status codes."""
from __future__ import annotations

import ctypes
import re
import subprocess
from pathlib import Path

import pytest

from mxmoe_amd import _native as nat

ROOT = Path(__file__).resolve().parent.parent
HEADERS = sorted((ROOT / "include").glob("*.h"))


def header_functions() -> set:
    txt = "\n".join(h.read_text() for h in HEADERS)
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return set(re.findall(r"^\s*(?:const\s+)?\w+\s*\*?\s*(\w+)\s*\(", txt, flags=re.M)) - {"defined"}


def test_header_lists_all_python_bound_symbols():
    assert header_functions() == set(nat.EXPORTED_SYMBOLS)


def test_library_exports_every_header_symbol():
    lib = nat.lib()
    for name in header_functions():
        assert hasattr(lib, name), name
    out = subprocess.run(["nm", "-D", "--defined-only", str(nat.LIB_PATH)], capture_output=True, text=True).stdout
    exported = {ln.split()[-1] for ln in out.splitlines() if " T " in ln}
    assert header_functions() <= exported


def test_struct_layouts():
    assert ctypes.sizeof(nat.MxmoeQParams) == 16  # QParams: 16-B stride, as int2+int+bool (8-B aligned)
    assert ctypes.sizeof(nat.MxmoeDim3) == 12
    assert ctypes.sizeof(nat.GGProblemC) == 5 * 8 + 8 * 4 + 3 * 8


def test_abi_version_and_variants():
    assert nat.lib().mxmoe_gg_abi_version() == nat.ABI_VERSION == 7
    vs = nat.list_variants()
    assert len(vs) == nat.variant_count() >= 1
    assert "w8a8_g-1_sym=TileConfig(" in vs[0]
    t = nat.variant_tile(0, 8, 8)
    assert t["BM"] > 0 and t["BN"] > 0 and t["threads"] % 64 == 0


def test_variant_caps_silu_epilogue():
    """mxmoe_gg_variant_caps (ABI 7): every product kernel carries the fused SiLU epilogue — v2x, v3,
    and (round 6) the small-batch wo3 kernel's fp16 / w8a8 / w4a4 bodies — what MoEFFN.gate_up_call
    asks instead of matching names."""
    names = {ln.split()[1]: int(ln.split()[0]) for ln in nat.list_variants()}
    assert set(names) >= {"v2x_256x256_w8_b3_buf_spread_edma", "v3_256x128_w4_dma_ring3_2wg", "wo3_64x256_w8_3wg"}
    for name, v in names.items():
        caps = nat.variant_caps(v)
        assert caps & nat.CAP_SILU_MUL, name
    with pytest.raises(nat.GGError):
        nat.variant_caps(len(names))


def test_stale_library_abi_refused(monkeypatch):
    """A library whose ABI version differs from the binding's raises NativeLibraryError at load (not an
    AttributeError later); a library named by MXMOE_GG_LIB (the A/B tools' older builds) may be
    older, down to ABI 5."""
    class Fn:
        def __init__(self, v):
            self.v = v

        def __call__(self):
            return self.v

    class Lib:
        def __init__(self, v):
            self.mxmoe_gg_abi_version = Fn(v)

    monkeypatch.delenv("MXMOE_GG_LIB", raising=False)
    nat._check_abi(Lib(nat.ABI_VERSION), nat.LIB_PATH)
    with pytest.raises(nat.NativeLibraryError):
        nat._check_abi(Lib(nat.ABI_VERSION - 1), nat.LIB_PATH)
    monkeypatch.setenv("MXMOE_GG_LIB", "/elsewhere/libmxmoe_gg_old.so")
    nat._check_abi(Lib(6), nat.LIB_PATH)
    with pytest.raises(nat.NativeLibraryError):
        nat._check_abi(Lib(nat.ABI_VERSION + 1), nat.LIB_PATH)
    with pytest.raises(nat.NativeLibraryError):
        nat._check_abi(object(), nat.LIB_PATH)


def test_workspace_size_grows_with_tiles():
    def ws(ps, v=0):
        arr = (nat.GGProblemC * len(ps))(*ps)
        return nat.workspace_size(arr, len(ps), v)

    small = ws([_prob(M=64)])
    big = ws([_prob(M=8192, N=4096)])
    assert 0 < small < big
    assert ws([_prob(M=0)]) > 0  # empty problems plan to an empty tile table


def test_struct_plan_info_layout():
    assert ctypes.sizeof(nat.GGPlanInfo) == 8 * 4 + 8 + 8 + 8 + 8  # + the plan signature, tile_slots


def test_auto_variant_follows_quant_mix():
    """MXMOE_GG_VARIANT_AUTO: only w4a4 -> the 256x128 variant, else the default (256x256)."""
    names = [ln.split()[1] for ln in nat.list_variants()]
    int4_v = names.index("v3_256x128_w4_dma_ring3_2wg")

    def ws(ps, v):
        arr = (nat.GGProblemC * len(ps))(*ps)
        return nat.workspace_size(arr, len(ps), v)

    assert names[nat.default_variant()] == "v2x_256x256_w8_b3_buf_spread_edma"
    big = dict(M=4096, N=4096, K=1024)
    w8 = [_prob(**big)]
    w4 = [_prob(a_bits=4, w_bits=4, **big)] * 2
    mix = [_prob(**big), _prob(a_bits=4, w_bits=4, **big)]
    assert ws(w8, nat.VARIANT_AUTO) == ws(w8, nat.default_variant())
    assert ws(mix, nat.VARIANT_AUTO) == ws(mix, nat.default_variant())
    assert ws(w4, nat.VARIANT_AUTO) == ws(w4, int4_v) != ws(w4, nat.default_variant())
    # an empty problem of another type does not count
    assert ws(w4 + [_prob(M=0)], nat.VARIANT_AUTO) == ws(w4 + [_prob(M=0)], int4_v)


def test_auto_variant_is_v2x_at_every_k():
    """AUTO (round 3): every call with fp16 / int8 problems runs v2x, at short and long K alike (v2x
    carries the 3-stage B ring that round 2's short-K rule chose v2s3 for)."""
    def auto(ps):
        arr = (nat.GGProblemC * len(ps))(*ps)
        return nat.resolve_variant(arr, len(ps))

    f16 = dict(a_bits=16, w_bits=16, scale_a=0, scale_b=0)
    for K in (256, 1408, 2048, 4096):
        assert auto([_prob(M=4096, N=4096, K=K, **f16)]) == nat.default_variant()
        assert auto([_prob(M=4096, N=4096, K=K)]) == nat.default_variant()
    from mxmoe_amd.workload import load_workload, qwen2_layer11_workload

    for bs in (8192, 2048):
        layer = load_workload(qwen2_layer11_workload(bs))["layer-11"]
        for gg in ("gate_up", "down"):
            probs = [_prob(M=s.M, N=s.N, K=s.K, **f16) for s in layer[gg]]
            assert auto(probs) == nat.default_variant(), (bs, gg)


def test_auto_variant_mid_batch_follows_k_skew():
    """The small-batch limit doubles for K-skewed calls (longest K >= 2x the weighted mean K): the
    qwen2_moe down call (shared expert K = 5632 vs 1408 routed) stays on wo3 up to bs 1024 (fp16 /
    w8a8) and 1536 (with int4), its gate_up call only to bs 512 / 768 (profiles/r03/wo2/wo3_mid.jsonl)."""
    names = [ln.split()[1] for ln in nat.list_variants()]
    wo3 = names.index("wo3_64x256_w8_3wg")

    def auto(ps):
        arr = (nat.GGProblemC * len(ps))(*ps)
        return nat.resolve_variant(arr, len(ps))

    from mxmoe_amd.workload import load_workload, qwen2_layer11_workload

    f16 = dict(a_bits=16, w_bits=16, scale_a=0, scale_b=0)
    for kw, qkw, gu_max, dn_max in ((f16, {}, 512, 1024), ({}, {"qstr": "w8a8_g-1_sym"}, 512, 1024),
                                    (dict(a_bits=4, w_bits=4), {"qstr": "w4a4_g-1_sym"}, 768, 1536)):
        for bs in (512, 768, 1024, 1536, 2048):
            layer = load_workload(qwen2_layer11_workload(bs, **qkw))["layer-11"]
            for gg, lim in (("gate_up", gu_max), ("down", dn_max)):
                v = auto([_prob(M=s.M, N=s.N, K=s.K, **kw) for s in layer[gg]])
                assert (v == wo3) == (bs <= lim), (qkw, bs, gg, names[v])


def test_auto_variant_small_batch_fp16_w8a8_runs_wo3():
    """AUTO (round 3): fp16 / w8a8 / w4a4 calls without weight-only problems take wo3 (64 x 128 tiles,
    3 WG per CU) while the weight-bytes-weighted mean M is <= 128 rows (qwen2_moe layer 11 at bs 128 /
    512), the general kernels from bs 2048 on; a bf16 / E4M3 / w4a4-g128 problem keeps them too."""
    names = [ln.split()[1] for ln in nat.list_variants()]
    wo3 = names.index("wo3_64x256_w8_3wg")

    def auto(ps):
        arr = (nat.GGProblemC * len(ps))(*ps)
        return nat.resolve_variant(arr, len(ps))

    from mxmoe_amd.workload import load_workload, qwen2_layer11_workload

    f16 = dict(a_bits=16, w_bits=16, scale_a=0, scale_b=0)
    for kw, qstr in ((f16, "fp16"), ({}, "w8a8_g-1_sym")):
        for bs, want in ((128, wo3), (512, wo3), (2048, nat.default_variant()), (8192, nat.default_variant())):
            layer = load_workload(qwen2_layer11_workload(bs, **({} if qstr == "fp16" else {"qstr": qstr})))["layer-11"]
            for gg in ("gate_up", "down"):
                probs = [_prob(M=s.M, N=s.N, K=s.K, **kw) for s in layer[gg]]
                assert auto(probs) == want, (qstr, bs, gg)
                w4 = _prob(M=8, N=256, K=layer[gg][0].K, a_bits=4, w_bits=4)
                assert auto(probs + [w4]) == want, (qstr, bs, gg)  # w4a4 rides along
                bf = _prob(M=8, N=256, K=layer[gg][0].K, a_bits=16, w_bits=16, scale_a=0, scale_b=0, fmt=nat.FMT_BF16)
                assert auto(probs + [bf]) == nat.default_variant(), (qstr, bs, gg)  # no bf16 body in wo3
    for bs, want in ((128, wo3), (512, wo3), (2048, None), (8192, None)):  # int4-only: v3 at large batch
        layer = load_workload(qwen2_layer11_workload(bs, qstr="w4a4_g-1_sym"))["layer-11"]
        for gg in ("gate_up", "down"):
            v = auto([_prob(M=s.M, N=s.N, K=s.K, a_bits=4, w_bits=4) for s in layer[gg]])
            assert (v == wo3) == (want == wo3), (bs, gg, v)


def test_auto_variant_weightonly_small_batch_runs_wo3():
    """AUTO (round 3): a call of weight-only problems (w8a8 problems may ride along: the reference's
    small-batch w4a16 + w8a8 pairing) runs wo3 (64-row tiles, 3 workgroups per CU) while the
    weight-bytes-weighted mean M is <= 512 rows, v2x above; int4 problems in the call keep the
    general kernels (wo3 has no int4 tile body)."""
    names = [ln.split()[1] for ln in nat.list_variants()]
    wo3 = names.index("wo3_64x256_w8_3wg")

    def auto(ps):
        arr = (nat.GGProblemC * len(ps))(*ps)
        return nat.resolve_variant(arr, len(ps))

    from mxmoe_amd.workload import load_workload, qwen2_layer11_workload

    for qstr in ("w4a16_g128_asym", "w4a16_g-1_sym", "w8a16_g-1_asym", "w2a16_g128_asym"):
        bits, g, sym = int(qstr[1]), int(qstr.split("_g")[1].split("_")[0]), qstr.endswith("_sym")
        wo = dict(a_bits=16, w_bits=bits, gsize=g, sym=int(sym), scale_a=0)
        for bs, want in ((128, wo3), (512, wo3), (2048, wo3), (8192, nat.default_variant())):
            layer = load_workload(qwen2_layer11_workload(bs, qstr=qstr))["layer-11"]
            for gg in ("gate_up", "down"):
                probs = [_prob(M=s.M, N=s.N, K=s.K, **wo) for s in layer[gg]]
                assert auto(probs) == want, (qstr, bs, gg)
                K = layer[gg][0].K
                assert auto(probs + [_prob(M=64, N=256, K=K)]) == want, (qstr, bs, gg)  # + a w8a8 problem
                f16 = _prob(M=64, N=256, K=K, a_bits=16, w_bits=16, scale_a=0, scale_b=0)
                assert auto(probs + [f16]) == want, (qstr, bs, gg)  # fp16 rides along too
                assert auto(probs + [_prob(M=64, N=256, K=K, a_bits=4, w_bits=4)]) == want  # w4a4 too
                g128 = _prob(M=64, N=256, K=K, a_bits=4, w_bits=4, gsize=128)
                assert auto(probs + [g128]) == nat.default_variant()  # no w4a4-g128 body in wo3
    assert auto([_prob(M=4096, N=256, K=1024)]) == nat.default_variant()  # w8a8 alone, large M: v2x
    assert not nat.variant_supports(wo3, "w4a4_g128_sym") and not nat.variant_supports(wo3, "bf16")
    assert all(nat.variant_supports(wo3, q) for q in ("fp16", "w8a8_g-1_sym", "w4a4_g-1_sym"))
    assert wo3 in nat.production_variants() and wo3 in nat.production_variants("w4a16_g128_asym")


def test_full_size_parity_covers_auto_choices():
    """Guard: the full-size parity parametrisation must contain the default
    variant and every variant AUTO resolves to on BASELINE configs[1]-[4], so a change to the
    product table cannot silently drop the kernel the bench times from the bs=8192 oracle checks."""
    from tests._util import FULL_SIZE_CFGS, full_size_layer, full_size_variants

    covered = set(full_size_variants())
    assert nat.default_variant() in covered
    for cfg in FULL_SIZE_CFGS:
        for gg, shapes in full_size_layer(cfg).items():
            probs = [_prob(M=s.M, N=s.N, K=s.K, a_bits=s.a_bits, w_bits=s.w_bits, gsize=s.gsize, sym=int(s.sym),
                           **({} if s.a_bits < 16 else dict(scale_a=0, scale_b=0))) for s in shapes]
            v = nat.resolve_variant((nat.GGProblemC * len(probs))(*probs), len(probs))
            assert v in covered, (cfg, gg, v)


def _plan(problems, ws_bytes=1 << 20):
    arr = (nat.GGProblemC * len(problems))(*problems)
    info = nat.GGPlanInfo()
    st = nat.lib().mxmoe_gg_plan(arr, len(problems), 0, None, ws_bytes, None, ctypes.byref(info))
    return st, nat.lib().mxmoe_gg_last_error().decode()


def _prob(**kw):
    d = dict(A=16, B=16, scale_a=16, scale_b=16, C=16, M=64, N=128, K=256, a_bits=8, w_bits=8, gsize=-1, sym=1)
    d.update(kw)
    return nat.GGProblemC(**d)


@pytest.mark.parametrize("kw,status,msg", [
    (dict(a_bits=4, w_bits=16, sym=0), nat.MXMOE_GG_ERR_UNSUPPORTED, "quant type not supported"),
    (dict(gsize=128), nat.MXMOE_GG_ERR_UNSUPPORTED, "quant type not supported"),
    (dict(K=24), nat.MXMOE_GG_ERR_INVALID, "multiple of 16"),
    (dict(N=100), nat.MXMOE_GG_ERR_INVALID, "multiple of 8"),
    (dict(M=-1), nat.MXMOE_GG_ERR_INVALID, "negative"),
    (dict(A=0), nat.MXMOE_GG_ERR_INVALID, "NULL"),
    (dict(scale_b=0), nat.MXMOE_GG_ERR_INVALID, "NULL scale"),
    (dict(C=8), nat.MXMOE_GG_ERR_INVALID, "aligned"),
    (dict(ldc=100), nat.MXMOE_GG_ERR_INVALID, "ldc"),
    (dict(K=262144), nat.MXMOE_GG_ERR_INVALID, "exact int32"),
])
def test_plan_validation(kw, status, msg):
    st, err = _plan([_prob(), _prob(**kw)])
    assert st == status
    assert msg in err and "problem 1" in err


def test_plan_needs_workspace():
    st, err = _plan([_prob()], ws_bytes=0)
    assert st == nat.MXMOE_GG_ERR_WORKSPACE and "workspace" in err


def test_fp16_problem_needs_no_scales():
    st, err = _plan([_prob(a_bits=16, w_bits=16, scale_a=0, scale_b=0)], ws_bytes=0)
    assert st == nat.MXMOE_GG_ERR_WORKSPACE  # passed validation, stopped at the workspace check


def test_missing_library_fails_loudly(monkeypatch, tmp_path):
    monkeypatch.setattr(nat, "_lib", None)
    monkeypatch.setenv("MXMOE_GG_LIB", str(tmp_path / "nope.so"))
    with pytest.raises(nat.NativeLibraryError):
        nat.lib()
    monkeypatch.setattr(nat, "_lib", None)


def test_splitk_planning():
    """A lone long-K problem (one CU's worth of tiles) is split along K on the v2 kernels: the
    workspace grows by the partial slabs; a full bs=8192 layer call is never split."""
    def ws(ps, v):
        arr = (nat.GGProblemC * len(ps))(*ps)
        return nat.workspace_size(arr, len(ps), v)

    names = [ln.split()[1] for ln in nat.list_variants()]
    v2s, v3 = nat.default_variant(), names.index("v3_256x128_w4_dma_ring3_2wg")
    lone = [_prob(M=512, N=2048, K=5632, a_bits=16, w_bits=16, scale_a=0, scale_b=0)]
    assert ws(lone, v2s) > ws(lone, v3) + 16 * 256 * 1024  # >= 2 slices x 16 tiles x 256 KiB slabs
    from mxmoe_amd.workload import load_workload, qwen2_layer11_workload

    layer = load_workload(qwen2_layer11_workload(8192))["layer-11"]["down"]
    probs = [_prob(M=s.M, N=s.N, K=s.K, a_bits=16, w_bits=16, scale_a=0, scale_b=0) for s in layer]
    assert ws(probs, v2s) < 1 << 20  # table only


def test_product_library_rejects_fp6_images():
    """MXMOE_GG_FMT_F6 (w4a4 as fp6 images) is a lab-library route: the
    product library refuses the format instead of running it."""
    p = nat.GGProblemC(A=16, B=16, scale_a=16, scale_b=16, C=16, M=64, N=256, K=256, a_bits=4, w_bits=4, gsize=-1,
                       sym=1, fmt=nat.FMT_F6, lda=0, ldb=0, ldc=0)
    arr = (nat.GGProblemC * 1)(p)
    with pytest.raises(nat.GGError, match="unknown operand format"):
        nat.workspace_size(arr, 1, nat.VARIANT_AUTO)
