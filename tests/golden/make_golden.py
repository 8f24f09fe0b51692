"""Generate the committed golden fixtures under tests/golden/ (and the LP-derived qconfig).

Runs ONLY in the build container, where /root/reference exists; the GPU box never runs it.
It imports the reference's own Python (SeaCatComplexes/MxMoE) from a /tmp copy (module import
writes into the source tree, compose_kernel.py:556), with two shims that change no arithmetic:
``enum.StrEnum`` (Python 3.10 lacks it; compose_kernel.py:6) and a pass-through ``jsbeautifier``
(formatting only; gen_workload.py:5). What the reference pins:

  quant_golden.npz ....... quant_minmax(t, bits, -1, True) on seeded fp16 rows (quant.py:40-84)
  qcfg_list_golden.json .. run_mxmoe_gg.get_qcfg_list on sample qconfig files (run_mxmoe_gg.py:11-29)
  variants_golden.json ... TemplateGenerator("89", qcfgs, Fused) variant enumeration + smem sizes
                           (compose_kernel.py:87-132, tile_config.py:266-286)
  workload_golden.json ... generate_workload_from_gate_trace outputs (gen_workload.py:38-110)
  tile_repr_golden.json .. the exporter's repr of TileConfig tuples (bits_solver.py:30,67-68)
  quant_g128_golden.npz .. quant_minmax(t, 4, 128, True) (group quantisation, quant.py:40-84)
  gg_w4a4g128_small.npz .. w4a4_g128_sym vectors (inputs by quant_minmax gsize 128, expected C by an
                           independent numpy restatement of the per-group fold, cta_gemm.cuh:610-772)
  gg_<kind>_small.npz .... GroupGEMM vectors: inputs quantised by the reference's quant_minmax,
                           packed per pack_wxax (quantize.cuh:425-475), expected C from an
                           independent numpy restatement (int64 matmul + epilogue mm_tile.cuh:469-496),
                           plus the reference-as-written column-scale permutation (mm_tile.cuh:452,462)
The LP-derived mixed qconfig is solved exactly (0/1 knapsack DP) from bits_model-1.lp.

  gg_fakequant_ref.npz ... the reference's OWN definition of a quantised linear, executed: for every
                           problem of the gg_*_small vectors, C_fq = F.linear(Quantizer.fake_quant(a),
                           Quantizer.fake_quant(b)) in fp32 (quant.py:87-106); plus weight-only
                           vectors (w2/w4/w8 a16, g-1 / g128, sym / asym): fp16 A, B, the reference's
                           quant_minmax codes / scales / zero points of B and
                           C_fq = F.linear(A, Quantizer(bits, sym, gsize).fake_quant(B))

Usage: python tests/golden/make_golden.py [--only-g128 | --only-fq]
"""
from __future__ import annotations

import enum
import json
import os
import re
import shutil
import sys
import types
from pathlib import Path

import numpy as np
import torch

HERE = Path(__file__).resolve().parent
ROOT = HERE.parent.parent
REF = Path("/root/reference")
TMP = Path("/tmp/mxmoe_ref_copy")


def import_reference():
    if TMP.exists():
        shutil.rmtree(TMP)
    shutil.copytree(REF, TMP, ignore=shutil.ignore_patterns("media"))

    class StrEnum(str, enum.Enum):
        def __str__(self):
            return self.value

        def __format__(self, spec):
            return self.value.__format__(spec)

    enum.StrEnum = StrEnum
    jsb = types.ModuleType("jsbeautifier")
    jsb.default_options = lambda: types.SimpleNamespace(indent_size=2)
    jsb.beautify = lambda s, o=None: s
    sys.modules["jsbeautifier"] = jsb
    sys.path.insert(0, str(TMP))
    import run_mxmoe_gg  # noqa: F401
    from mxmoe.kernels import compose_kernel, gen_workload, tile_config
    from mxmoe.quant.quant import Quantizer, quant_minmax
    return types.SimpleNamespace(quant_minmax=quant_minmax, Quantizer=Quantizer, get_qcfg_list=run_mxmoe_gg.get_qcfg_list,
                                 compose_kernel=compose_kernel, tile_config=tile_config, gen_workload=gen_workload)


# ------------------------------------------------------------------ LP -> mixed qconfig

def solve_lp1(lp_path: Path):
    """Exact solve of bits_model-1.lp: min sum c*x, budget <= 960, gate==up tie, one strategy each."""
    txt = lp_path.read_text()
    obj_txt = txt.split("Minimize")[1].split("Subject To")[0]
    cost = {}
    for c, e, w, s in re.findall(r"([-+]?\d+(?:\.\d+)?(?:e[-+]?\d+)?) x\[(\d+),(\d+),(\d+)\]", obj_txt):
        cost[(int(e), int(w), int(s))] = float(c)
    bud_txt = txt.split("memory_budget:")[1].split("<=")
    cap = int(float(bud_txt[1].split()[0]))
    bits = {}
    for c, e, w, s in re.findall(r"(\d+) x\[(\d+),(\d+),(\d+)\]", bud_txt[0]):
        bits[(int(e), int(w), int(s))] = int(c)
    E = 1 + max(e for e, _, _ in cost)
    # items: (e, "gu") with gate+up tied, (e, "down")
    base_bits = sum(bits[(e, w, 0)] for e in range(E) for w in range(3))
    base_cost = sum(cost[(e, w, 0)] for e in range(E) for w in range(3))
    unit = 4
    capu = (cap - base_bits) // unit
    items = []
    for e in range(E):
        wgt = (bits[(e, 0, 1)] - bits[(e, 0, 0)] + bits[(e, 1, 1)] - bits[(e, 1, 0)]) // unit
        gain = cost[(e, 0, 0)] - cost[(e, 0, 1)] + cost[(e, 1, 0)] - cost[(e, 1, 1)]
        items.append(((e, "gu"), wgt, gain))
        wgt = (bits[(e, 2, 1)] - bits[(e, 2, 0)]) // unit
        gain = cost[(e, 2, 0)] - cost[(e, 2, 1)]
        items.append(((e, "down"), wgt, gain))
    # 0/1 knapsack maximising gain
    best = np.full(capu + 1, -np.inf)
    best[0] = 0.0
    take = np.zeros((len(items), capu + 1), dtype=bool)
    for i, (_, wgt, gain) in enumerate(items):
        new = best.copy()
        for c in range(capu, wgt - 1, -1):
            if best[c - wgt] + gain > new[c]:
                new[c] = best[c - wgt] + gain
                take[i, c] = True
        best = new
    c = int(np.argmax(best))
    chosen = set()
    for i in range(len(items) - 1, -1, -1):
        if take[i, c]:
            chosen.add(items[i][0])
            c -= items[i][1]
    used = sum(w for (k, w, _) in items if k in chosen) * unit
    obj = base_cost - float(np.max(best))
    return E, chosen, used, obj


def make_lp_qconfig(ref) -> dict:
    E, chosen, used, obj = solve_lp1(REF / "bits_model-1.lp")
    w8 = "w8a8_g-1_sym"
    w4 = "w4a4_g-1_sym"
    strat = {11: {e: {0: w8 if (e, "gu") in chosen else w4, 1: w8 if (e, "gu") in chosen else w4,
                      2: w8 if (e, "down") in chosen else w4} for e in range(E)}}
    from mxmoe_amd.qconfig import export_qconfig

    qc = export_qconfig(strat)
    meta = {"E": E, "extra_bits_used": used, "objective": round(obj, 4),
            "w8a8_gate_up": sorted(e for (e, k) in chosen if k == "gu"),
            "w8a8_down": sorted(e for (e, k) in chosen if k == "down")}
    return qc, meta


# ------------------------------------------------------------------ GroupGEMM vectors

def pack_np(q: np.ndarray, bits: int) -> np.ndarray:
    """Independent numpy restatement of pack_wxax (quantize.cuh:425-475)."""
    rows, K = q.shape
    pack = 16 // bits
    words = np.zeros((rows, K // pack), dtype=np.uint16)
    mask = (1 << bits) - 1
    for x in range(pack):
        field = (q[:, x::pack].astype(np.int16) & mask).astype(np.uint16)
        words |= field << np.uint16((pack - 1 - x) * bits)
    return words.view(np.uint8).reshape(rows, K * bits // 8)


def epilogue_np(acc: np.ndarray, sa: np.ndarray, sb: np.ndarray, sb_cols: np.ndarray | None = None) -> np.ndarray:
    sbv = sb if sb_cols is None else sb[sb_cols]
    s16 = (sa.astype(np.float32)[:, None] * sbv.astype(np.float32)[None, :]).astype(np.float16)
    return (np.float32(0) + acc.astype(np.float32) * s16.astype(np.float32)).astype(np.float16)


def ref_bug_cols(N: int) -> np.ndarray:
    """Column the reference-as-written reads sb from (mm_tile.cuh:452,462-463 vs :633):
    the C fragment holds cols 8*(c//8) + 2*(lane%4) + {0,1}, load_scale reads lane%4 + {0,1}."""
    c = np.arange(N)
    return 8 * (c // 8) + (c % 8) // 2 + (c % 2)


def make_gg_vectors(ref, kind: str, specs, seed: int) -> dict:
    g = torch.Generator().manual_seed(seed)
    out = {"P": np.int32(len(specs))}
    for i, (M, N, K, q) in enumerate(specs):
        a = (torch.rand(M, K, generator=g) * 2 - 1).half()
        b = (torch.rand(N, K, generator=g) * 2 - 1).half()
        out[f"p{i}_shape"] = np.array([M, N, K], np.int32)
        if q == "fp16":
            out[f"p{i}_bits"] = np.int32(16)
            out[f"p{i}_A"] = a.numpy()
            out[f"p{i}_B"] = b.numpy()
            out[f"p{i}_C_f64"] = (a.double() @ b.double().T).numpy()
            continue
        bits = 8 if q == "w8a8_g-1_sym" else 4
        qa, sa, _ = ref.quant_minmax(a, bits, -1, True)
        qb, sb, _ = ref.quant_minmax(b, bits, -1, True)
        qa = qa.to(torch.int8).numpy()
        qb = qb.to(torch.int8).numpy()
        sa = sa.reshape(-1).numpy().astype(np.float16)
        sb = sb.reshape(-1).numpy().astype(np.float16)
        acc = qa.astype(np.int64) @ qb.astype(np.int64).T
        out[f"p{i}_bits"] = np.int32(bits)
        out[f"p{i}_qa"], out[f"p{i}_qb"] = qa, qb
        out[f"p{i}_A"], out[f"p{i}_B"] = pack_np(qa, bits), pack_np(qb, bits)
        out[f"p{i}_sa"], out[f"p{i}_sb"] = sa, sb
        out[f"p{i}_acc"] = acc
        out[f"p{i}_C"] = epilogue_np(acc, sa, sb)
        out[f"p{i}_C_refbug"] = epilogue_np(acc, sa, sb, ref_bug_cols(N))
    return out


def fold_g128_np(qa: np.ndarray, qb: np.ndarray, sa: np.ndarray, sb: np.ndarray, gsize: int) -> np.ndarray:
    """Independent numpy restatement of the w4a4 g128 epilogue (cta_gemm.cuh:610-772, mm_tile.cuh:490-493):
    out = fma(f32(acc_g), f32(fp16(sa_g * sb_g)), out) per group in order, C = fp16(out). The fma is
    formed in f64 (the product is exact there) and the f64 sum is checked exact by TwoSum, so the one
    f32 rounding below is the fma's single rounding."""
    M, K = qa.shape
    N = qb.shape[0]
    G = K // gsize
    out = np.zeros((M, N), np.float32)
    for g in range(G):
        ks = slice(g * gsize, (g + 1) * gsize)
        acc = qa[:, ks].astype(np.int64) @ qb[:, ks].astype(np.int64).T
        s16 = (sa[g * M:(g + 1) * M].astype(np.float32)[:, None] *
               sb[g * N:(g + 1) * N].astype(np.float32)[None, :]).astype(np.float16)
        p = acc.astype(np.float64) * s16.astype(np.float64)
        o = out.astype(np.float64)
        t = p + o
        bp = t - o
        err = (p - bp) + (o - (t - bp))
        assert (err == 0).all(), "f64 sum not exact: the restatement would double-round"
        out = t.astype(np.float32)
    return out.astype(np.float16)


def make_g128_vectors(ref, specs, seed: int) -> dict:
    """w4a4_g128_sym vectors: inputs quantised by the reference's quant_minmax(t, 4, 128, True)
    (scales [rows*K/128] in (row, group) order, then permute_scale -> [K/128][rows])."""
    g = torch.Generator().manual_seed(seed)
    out = {"P": np.int32(len(specs))}
    for i, (M, N, K) in enumerate(specs):
        a = (torch.rand(M, K, generator=g) * 2 - 1).half()
        b = (torch.rand(N, K, generator=g) * 2 - 1).half()
        qa, sa, _ = ref.quant_minmax(a, 4, 128, True)
        qb, sb, _ = ref.quant_minmax(b, 4, 128, True)
        qa, qb = qa.to(torch.int8).numpy(), qb.to(torch.int8).numpy()
        sa = np.ascontiguousarray(sa.reshape(M, K // 128).numpy().astype(np.float16).T).reshape(-1)
        sb = np.ascontiguousarray(sb.reshape(N, K // 128).numpy().astype(np.float16).T).reshape(-1)
        out[f"p{i}_shape"] = np.array([M, N, K], np.int32)
        out[f"p{i}_bits"] = np.int32(4)
        out[f"p{i}_qa"], out[f"p{i}_qb"] = qa, qb
        out[f"p{i}_A"], out[f"p{i}_B"] = pack_np(qa, 4), pack_np(qb, 4)
        out[f"p{i}_sa"], out[f"p{i}_sb"] = sa, sb
        out[f"p{i}_C"] = fold_g128_np(qa, qb, sa, sb, 128)
    return out


def make_g128(ref):
    """quant_g128_golden.npz (quant_minmax gsize 128 on seeded rows) + gg_w4a4g128_small.npz."""
    qg = {}
    g = torch.Generator().manual_seed(4321)
    t = (torch.randn(17, 512, generator=g) * torch.logspace(-3, 1, 17)[:, None]).half()
    t[2, 128:256] = 0.001 * t[2, 128:256]  # one tiny group
    t[4, 300] = 9.0  # outlier inside one group
    q, s, _ = ref.quant_minmax(t, 4, 128, True)
    qg["x_4"] = t.numpy()
    qg["q_4"] = q.to(torch.int8).numpy()
    qg["scale_4"] = s.reshape(-1).numpy().astype(np.float16)  # (row, group) order, as quant_minmax returns
    np.savez_compressed(HERE / "quant_g128_golden.npz", **qg)
    specs = [(0, 256, 256), (1, 256, 128), (17, 128, 384), (130, 256, 1408), (257, 384, 256)]
    np.savez_compressed(HERE / "gg_w4a4g128_small.npz", **make_g128_vectors(ref, specs, seed=128))


# ------------------------------------------------------------------ reference-executed fake-quant C

FQ_SOURCES = {  # fixture -> (seed, specs) exactly as main() / make_g128() build them
    "w8a8": ("gg_w8a8_small.npz", 42), "w4a4": ("gg_w4a4_small.npz", 43), "mixed": ("gg_mixed_small.npz", 45),
    "w4a4g128": ("gg_w4a4g128_small.npz", 128)}

WO_SPECS = [  # (M, N, K, w_bits, gsize, sym): weight-only problems, A fp16
    (17, 128, 256, 4, -1, True), (130, 256, 384, 4, -1, False), (33, 128, 512, 4, 128, False),
    (64, 256, 256, 4, 128, True), (77, 128, 256, 8, -1, False), (9, 128, 384, 8, 128, False),
    (40, 256, 256, 8, -1, True), (21, 128, 512, 2, 128, False), (50, 128, 256, 2, -1, False),
    (1, 128, 1024, 4, 128, False)]


def make_fakequant(ref):
    """gg_fakequant_ref.npz: the reference's Quantizer.fake_quant (quant.py:87-106) run on the same
    seeded fp16 inputs as the committed GroupGEMM vectors, then F.linear in fp32. The codes of each
    regenerated input are first checked against the committed fixture (same seed stream)."""
    import torch.nn.functional as F

    out = {}
    for kind, (fname, seed) in FQ_SOURCES.items():
        d = np.load(HERE / fname)
        g = torch.Generator().manual_seed(seed)
        for i in range(int(d["P"])):
            M, N, K = (int(x) for x in d[f"p{i}_shape"])
            a = (torch.rand(M, K, generator=g) * 2 - 1).half()
            b = (torch.rand(N, K, generator=g) * 2 - 1).half()
            bits = int(d[f"p{i}_bits"])
            if bits == 16:
                continue
            gsize = 128 if kind == "w4a4g128" else -1
            qa, _, _ = ref.quant_minmax(a, bits, gsize, True)
            qb, _, _ = ref.quant_minmax(b, bits, gsize, True)
            assert (qa.to(torch.int8).numpy() == d[f"p{i}_qa"]).all() and (qb.to(torch.int8).numpy() == d[f"p{i}_qb"]).all()
            qz = ref.Quantizer(bits, True, gsize)
            cfq = F.linear(qz.fake_quant(a).float(), qz.fake_quant(b).float()) if M else torch.zeros(0, N)
            out[f"{kind}_p{i}_Cfq"] = cfq.numpy().astype(np.float32)
    g = torch.Generator().manual_seed(777)
    out["wo_P"] = np.int32(len(WO_SPECS))
    for i, (M, N, K, bits, gsize, sym) in enumerate(WO_SPECS):
        a = (torch.rand(M, K, generator=g) * 2 - 1).half()
        b = (torch.rand(N, K, generator=g) * 2 - 1).half()
        q, s, z = ref.quant_minmax(b, bits, gsize, sym)
        qz = ref.Quantizer(bits, sym, gsize)
        out[f"wo{i}_spec"] = np.array([M, N, K, bits, gsize, int(sym)], np.int32)
        out[f"wo{i}_A"], out[f"wo{i}_B"] = a.numpy(), b.numpy()
        out[f"wo{i}_q"] = q.to(torch.uint8 if not sym else torch.int8).numpy()
        G = 1 if gsize == -1 else K // gsize
        out[f"wo{i}_scale"] = s.reshape(N, G).numpy().astype(np.float16)
        out[f"wo{i}_zp"] = (np.zeros((N, G), np.float16) if sym else z.reshape(N, G).numpy().astype(np.float16))
        out[f"wo{i}_Cfq"] = F.linear(a.float(), qz.fake_quant(b).float()).numpy().astype(np.float32)
    np.savez_compressed(HERE / "gg_fakequant_ref.npz", **out)


def main():
    sys.path.insert(0, str(ROOT))
    ref = import_reference()
    if "--only-g128" in sys.argv:
        make_g128(ref)
        return
    if "--only-fq" in sys.argv:
        make_fakequant(ref)
        return
    torch.manual_seed(0)

    # 1. quant_minmax golden
    qg = {}
    g = torch.Generator().manual_seed(1234)
    for bits in (8, 4):
        t = (torch.randn(33, 256, generator=g) * torch.logspace(-3, 1, 33)[:, None]).half()
        t[3, :] = 0.001 * t[3, :]  # tiny row
        t[5, 7] = 7.5  # outlier
        q, s, _ = ref.quant_minmax(t, bits, -1, True)
        qg[f"x_{bits}"] = t.numpy()
        qg[f"q_{bits}"] = q.to(torch.int8).numpy()
        qg[f"scale_{bits}"] = s.reshape(-1).numpy().astype(np.float16)
    np.savez_compressed(HERE / "quant_golden.npz", **qg)

    # 2. LP-derived mixed qconfig (+ qcfg lists)
    qc, meta = make_lp_qconfig(ref)
    wl_dir = ROOT / "mxmoe_amd" / "workloads"
    with open(wl_dir / "qconfig_qwen2_moe_w4a4+w8a8_wbits5.0_lp1.json", "w") as f:
        json.dump(qc, f)
    with open(HERE / "lp1_solution.json", "w") as f:
        json.dump(meta, f, indent=1)
    qcfg_lists = {}
    tmpq = Path("/tmp/mxmoe_golden_qcfg.json")
    tmpq.write_text(json.dumps(qc))
    qcfg_lists["lp1_layer11"] = sorted(ref.get_qcfg_list(str(tmpq), 11))
    qcfg_lists["lp1_all"] = sorted(ref.get_qcfg_list(str(tmpq), -1))
    qcfg_lists["lp1_layer3"] = sorted(ref.get_qcfg_list(str(tmpq), 3))
    uni = {"0": {"experts": {"0": {k: {"w_bits": 4, "w_gsize": 128, "w_sym": False, "w_clip": [1, 1], "a_bits": 16,
                                       "a_gsize": -1, "a_sym": True, "a_clip": [1, 1]} for k in ("gate", "up", "down")}}},
           "LT": {"0": [1.0, 2.0]}}
    tmpq.write_text(json.dumps(uni))
    qcfg_lists["w4a16_asym"] = sorted(ref.get_qcfg_list(str(tmpq), -1))
    with open(HERE / "qcfg_list_golden.json", "w") as f:
        json.dump({"lists": qcfg_lists, "uniform_qconfig": uni}, f, indent=1)

    # 3. variant enumeration + smem (sm89 lists)
    ck = ref.compose_kernel
    var = {}
    for qs in (["fp16"], ["w8a8_g-1_sym"], ["w4a4_g-1_sym"], ["w4a4_g-1_sym", "w8a8_g-1_sym"]):
        gen = ck.TemplateGenerator("89", qs, ck.KernelType.Fused)
        combos = gen.get_tile_configs()
        var["+".join(qs)] = {
            "count": len(combos),
            "first": {k: v.to_str() for k, v in combos[0].items()},
            "smem": [list(gen.get_smem_size(c)) for c in combos],
            "tiles": [{k: [v.BM, v.BN, v.BK, v.WM, v.WN, v.WK, v.STAGE] for k, v in c.items()} for c in combos],
        }
    with open(HERE / "variants_golden.json", "w") as f:
        json.dump(var, f, indent=1)

    # 4. tile_cfg repr (exporter form)
    tc = ref.tile_config
    tiles = (tc.get_possible_tile_list("89", "w4a4_g-1_sym")[0], tc.get_possible_tile_list("89", "w8a8_g-1_sym")[2])
    tiles = tuple(ck.format_template(t, tc.QCFG_MAP[q]) for t, q in zip(tiles, ["w4a4_g-1_sym", "w8a8_g-1_sym"]))
    with open(HERE / "tile_repr_golden.json", "w") as f:
        json.dump({"tile_cfg_file": {"11": repr(tiles)},
                   "expected": [[t.BM, t.BN, t.BK, t.WM, t.WN, t.WK, t.STAGE, t.SPLITK, t.MMA] for t in tiles]}, f,
                  indent=1)

    # 5. workload generation
    from mxmoe_amd.workload import qwen2_layer11_trace

    trace = qwen2_layer11_trace()
    trace["layer-3"] = {"access_freq": list(range(1, 61))}
    tpath = Path("/tmp/mxmoe_golden_trace.json")
    tpath.write_text(json.dumps(trace))
    wls = {}
    tmpq.write_text(json.dumps(qc))
    for name, kw in {"fp16_8192_l11": dict(num_total_tokens=8192, layer_id=11),
                     "w8a8_512_all": dict(num_total_tokens=512, layer_id=-1, qstr="w8a8_g-1_sym"),
                     "lp1_8192_l11": dict(num_total_tokens=8192, layer_id=11, qcfg_file=str(tmpq)),
                     "fp16_128_l11": dict(num_total_tokens=128, layer_id=11)}.items():
        out = Path(f"/tmp/mxmoe_golden_wl_{name}.json")
        ref.gen_workload.generate_workload_from_gate_trace(str(tpath), save_path=str(out), **kw)
        wls[name] = {"args": {k: (v if k != "qcfg_file" else "LP1") for k, v in kw.items()},
                     "workload": json.loads(out.read_text())}
    with open(HERE / "workload_golden.json", "w") as f:
        json.dump({"trace": trace, "cases": wls}, f)

    # 6. GroupGEMM vectors
    edge = [(0, 128, 256), (1, 128, 256), (17, 256, 128), (130, 128, 384), (257, 256, 256)]
    np.savez_compressed(HERE / "gg_w8a8_small.npz",
                        **make_gg_vectors(ref, "w8a8", [(*s, "w8a8_g-1_sym") for s in edge], 42))
    np.savez_compressed(HERE / "gg_w4a4_small.npz",
                        **make_gg_vectors(ref, "w4a4", [(*s, "w4a4_g-1_sym") for s in edge], 43))
    np.savez_compressed(HERE / "gg_fp16_small.npz", **make_gg_vectors(ref, "fp16", [(*s, "fp16") for s in edge], 44))
    mixed = [(130, 256, 256, "w8a8_g-1_sym"), (0, 128, 128, "w4a4_g-1_sym"), (77, 128, 512, "w4a4_g-1_sym"),
             (33, 256, 128, "fp16"), (257, 128, 256, "w8a8_g-1_sym"), (9, 256, 1024, "w4a4_g-1_sym")]
    np.savez_compressed(HERE / "gg_mixed_small.npz", **make_gg_vectors(ref, "mixed", mixed, 45))
    make_g128(ref)
    make_fakequant(ref)
    print("golden fixtures written;", meta)


if __name__ == "__main__":
    main()
