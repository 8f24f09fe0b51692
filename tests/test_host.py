"""Host-logic tests (CPU): qconfig / tile_config / workload JSON surfaces vs the reference's outputs."""
from __future__ import annotations

import json
from pathlib import Path

import pytest

from mxmoe_amd import qconfig as qc
from mxmoe_amd import tile_config as tc
from mxmoe_amd import workload as wl

GOLD = Path(__file__).resolve().parent / "golden"


def test_get_qcfg_list_matches_reference():
    g = json.loads((GOLD / "qcfg_list_golden.json").read_text())
    lp = wl.mixed_qconfig_lp1()
    assert sorted(qc.get_qcfg_list(lp, 11)) == g["lists"]["lp1_layer11"]
    assert sorted(qc.get_qcfg_list(lp, -1)) == g["lists"]["lp1_all"]
    assert sorted(qc.get_qcfg_list(lp, 3)) == g["lists"]["lp1_layer3"]
    assert sorted(qc.get_qcfg_list(g["uniform_qconfig"], -1)) == g["lists"]["w4a16_asym"]


def test_lp1_mixed_qconfig_solution():
    sol = json.loads((GOLD / "lp1_solution.json").read_text())
    lp = wl.mixed_qconfig_lp1()
    experts = lp["11"]["experts"]
    assert len(experts) == 61
    gu8 = sorted(int(e) for e, c in experts.items() if c["gate"]["w_bits"] == 8)
    dn8 = sorted(int(e) for e, c in experts.items() if c["down"]["w_bits"] == 8)
    assert gu8 == sol["w8a8_gate_up"] and dn8 == sol["w8a8_down"]
    assert all(c["gate"] == c["up"] for c in experts.values())  # gate=up tie (bits_solver.py:378-379)
    # budget: 4 bits * 3 linears * 60 + 16 * 3 (shared) + upgrades <= 960 (bits_model-1.lp:188-261)
    bits = sum((4 if int(e) < 60 else 16) * (c[k]["w_bits"] // 4) for e, c in experts.items()
               for k in ("gate", "up", "down"))
    assert bits == 960 and sol["extra_bits_used"] == 192
    assert abs(sol["objective"] - 2212.48) < 0.01


@pytest.mark.parametrize("case", ["fp16_8192_l11", "w8a8_512_all", "lp1_8192_l11", "fp16_128_l11"])
def test_workload_generation_matches_reference(case):
    g = json.loads((GOLD / "workload_golden.json").read_text())
    c = g["cases"][case]
    args = dict(c["args"])
    T = args.pop("num_total_tokens")
    layer = args.pop("layer_id")
    kw = {}
    if "qstr" in args:
        kw["qstr"] = args["qstr"]
    if args.get("qcfg_file") == "LP1":
        kw["qconfig"] = wl.mixed_qconfig_lp1()
    ours = wl.generate_workload_from_trace(g["trace"], T, layer, **kw)
    assert json.loads(json.dumps(ours)) == c["workload"]


def test_layer11_workload_uses_committed_histogram():
    w = wl.load_workload(wl.qwen2_layer11_workload(8192))["layer-11"]
    h = wl.qwen2_hist()
    assert [p.M for p in w["gate_up"][:-1]] == h["M"]
    assert (w["gate_up"][-1].M, w["gate_up"][-1].N, w["gate_up"][-1].K) == (8192, 11264, 2048)
    assert (w["down"][-1].M, w["down"][-1].N, w["down"][-1].K) == (8192, 2048, 5632)
    gf = sum(p.flops for p in w["gate_up"]) / 1e9
    df = sum(p.flops for p in w["down"]) / 1e9
    assert abs(gf - 755.8) < 0.1 and abs(df - 377.9) < 0.1


def test_parse_workload_floats_to_int():
    d = {"num_tokens": 8, "layer-1": {"gate_up": [{"shape": [8, 11264.0, 2048], "w_bits": 16, "a_bits": 16,
                                                   "gsize": -1, "sym": True}], "down": []}}
    p = wl.load_workload(d)["layer-1"]["gate_up"][0]
    assert p.shape == [8, 11264, 2048] and p.qcfg == "fp16"


def test_tile_repr_parser_exporter_form():
    g = json.loads((GOLD / "tile_repr_golden.json").read_text())
    parsed = tc.parse_tile_config_json(g["tile_cfg_file"], ["w8a8_g-1_sym", "w4a4_g-1_sym"], layer=11)
    exp = g["expected"]
    got = [parsed["w4a4_g-1_sym"][0], parsed["w8a8_g-1_sym"][0]]
    for t, e in zip(got, exp):
        assert [t.BM, t.BN, t.BK, t.WM, t.WN, t.WK, t.STAGE, t.SPLITK, t.MMA] == e


def test_tile_repr_parser_never_evaluates():
    evil = {"1": "(TileConfig(BM=__import__('os').system('false'), BN=128), )"}
    parsed = tc.parse_tile_config_json(evil, ["fp16"], layer=1)
    assert parsed["fp16"][0].BN == 128 and parsed["fp16"][0].BM == 64  # BM field not an int literal -> default


def test_smem_formula_matches_reference_variant_table():
    g = json.loads((GOLD / "variants_golden.json").read_text())
    assert g["fp16"]["count"] == 5 and g["w8a8_g-1_sym"]["count"] == 6 and g["w4a4_g-1_sym"]["count"] == 5
    assert g["w4a4_g-1_sym+w8a8_g-1_sym"]["count"] == 30
    for key, bits in (("fp16", 16), ("w8a8_g-1_sym", 8), ("w4a4_g-1_sym", 4)):
        for tiles, smem in zip(g[key]["tiles"], g[key]["smem"]):
            (BM, BN, BK, WM, WN, WK, ST), = tiles.values()
            t = tc.TileConfig(BM=BM, BN=BN, BK=BK, WM=WM, WN=WN, WK=WK, STAGE=ST)
            assert t.smem_bytes_tile(bits, bits) == smem[0]
            assert t.smem_bytes_scale(bits < 16) == smem[1]


def test_qcfg_info():
    assert tc.get_info_from_qcfg_str("w8a8_g-1_sym") == (8, 8, -1, True)
    assert tc.get_info_from_qcfg_str("w4a16_g128_asym") == (4, 16, 128, False)
    assert set(tc.MI355X_QCFG) <= set(tc.SUPPORTED_QCFG)


def test_cli_workload_step(tmp_path, monkeypatch):
    import run_mxmoe_gg as cli

    class A:
        qconfig = str(wl.WORKLOAD_DIR / "qconfig_qwen2_moe_w4a4+w8a8_wbits5.0_lp1.json")
        qstr = None
        layer = 11

    suffix, kw, qcfgs = cli.workload_suffix(A)
    assert suffix == "-5.0_lp1.json" and qcfgs == ["w4a4_g-1_sym", "w8a8_g-1_sym"] and "qconfig" in kw
    A.qconfig, A.qstr = None, "w8a8_g-1_sym"
    assert cli.workload_suffix(A)[0] == "-w8a8_g-1_sym.json"
    A.qstr = None
    assert cli.workload_suffix(A)[0] == "-fp16.json"
    t = cli.find_trace("qwen2_moe", "wiki2", 11, None)
    assert t["topk"] == 4 and len(t["layer-11"]["access_freq"]) == 60 and len([k for k in t if k.startswith("layer-")]) == 24


def test_ds2_mixed_allocation_pinned():
    """DeepSeek-V2-Lite mixed config: seeded greedy w8a8 pick up to 25 % of units."""
    g = json.loads((GOLD / "ds2_mixed_alloc.json").read_text())
    ex = wl.ds2_mixed_qconfig()["1"]["experts"]
    assert len(ex) == 65 and all(c["gate"] == c["up"] for c in ex.values())
    assert sorted(int(e) for e, c in ex.items() if c["gate"]["w_bits"] == 8) == g["w8a8_gate_up"]
    assert sorted(int(e) for e, c in ex.items() if c["down"]["w_bits"] == 8) == g["w8a8_down"]
    units = sum((2 if e == "64" else 1) * (2 if lin == "gate" else 1)
                for e, c in ex.items() for lin in ("gate", "down") if c[lin]["w_bits"] == 8)
    assert units == g["units_w8a8"] <= 0.25 * (64 * 3 + 2 * 3)
    layer = wl.load_workload(wl.ds2_workload(8192, qconfig=wl.ds2_mixed_qconfig()))["layer-1"]
    assert sum(p.M for p in layer["gate_up"][:-1]) == 8192 * 6 and layer["gate_up"][-1].shape == [8192, 5632, 2048]
    assert layer["down"][-1].shape == [8192, 2048, 2816]


def test_cpu_plumbing_bs128_config0(tmp_path, monkeypatch):
    """BASELINE configs[0]: `run_mxmoe_gg.py --bs 128 --cpu-plumbing` writes the layer-11 workload
    (61 problems per GroupGEMM, shared expert last with M = 128, routed M_e = int(p_e * 128 * 4)) and
    times the per-problem torch.matmul fp16 path on the host — no GPU, no HIP kernel."""
    import json

    import run_mxmoe_gg as cli
    from mxmoe_amd.workload import qwen2_hist

    monkeypatch.setattr(cli, "CUR_DIR", str(tmp_path))
    out = cli.main(["--model", "qwen2_moe", "--bs", "128", "--layer", "11", "--cpu-plumbing"])
    assert [(gg, n) for _, gg, n, _ in out] == [("gate_up", 61), ("down", 61)]
    wl = json.load(open(tmp_path / "out" / "workloads" / "qwen2_moe-wiki2-128-fp16.json"))
    gate_up = wl["layer-11"]["gate_up"]
    assert gate_up[-1]["shape"] == [128, 11264, 2048]
    h = qwen2_hist()["M"]
    tot = sum(h)
    assert [p["shape"][0] for p in gate_up[:-1]] == [int(m / tot * 128 * 4) for m in h]
    assert (tmp_path / "out" / "bench" / "qwen2_moe-wiki2-128-fp16-layer-11-gate_up-cpu.csv").exists()


def test_other_model_workloads_follow_gen_workload_rules():
    """mixtral / qwen2_moe_57b (gen_workload.py:16-21; MODEL_SHAPES) with seeded synthetic routing:
    routed M_e = int(p_e * T * topk), shared expert last (none for mixtral), gate_up N = 2 * N_e."""
    from mxmoe_amd.workload import MODEL_SHAPES, load_workload, model_workload, synthetic_trace

    for model in ("mixtral", "qwen2_moe_57b"):
        s = MODEL_SHAPES[model]
        wl = load_workload(model_workload(model, 4096, qstr="w8a8_g-1_sym_E4M3"))["layer-1"]
        t = synthetic_trace(model, 4096)
        freq = t["layer-1"]["access_freq"]
        assert sum(freq) == 4096 * s["topk"]
        n_shared = 1 if s["S"] else 0
        assert len(wl["gate_up"]) == s["E"] + n_shared and len(wl["down"]) == s["E"] + n_shared
        for e, p in enumerate(wl["gate_up"][: s["E"]]):
            assert p.shape == [int(freq[e] / sum(freq) * 4096 * s["topk"]), 2 * s["N"], s["K"]]
            assert p.qcfg == "w8a8_g-1_sym_E4M3"
        if n_shared:
            assert wl["gate_up"][-1].shape == [4096, int(2 * s["N"] * s["S"]), s["K"]]
            assert wl["down"][-1].shape == [4096, s["K"], int(s["N"] * s["S"])]
