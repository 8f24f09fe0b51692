"""The reference CLI surface on the GPU: run_mxmoe_gg.main in --mode check (every sampled output
against the CPU recomputation of mxmoe_amd/check.py) for a mixed qconfig with an exporter-form
tile_config, a weight-only qstr and w4a4 g128; CSV schema kernel_name,avg_time,TFLOPS,speedup
(test.cu:855-865); tile_config -> variant mapping (tile_config.select_variant)."""
from __future__ import annotations

import csv
import json
from pathlib import Path

import pytest

import run_mxmoe_gg
from mxmoe_amd import _native as nat

pytestmark = pytest.mark.gpu
GOLD = Path(__file__).resolve().parent / "golden"
LP1 = Path(run_mxmoe_gg.ROOT) / "mxmoe_amd" / "workloads" / "qconfig_qwen2_moe_w4a4+w8a8_wbits5.0_lp1.json"


@pytest.fixture
def out_dir(tmp_path, monkeypatch):
    monkeypatch.setattr(run_mxmoe_gg, "CUR_DIR", str(tmp_path))
    return tmp_path


def _csv_ok(paths, n_rows):
    assert len(paths) == 2  # gate_up and down
    for p in paths:
        with open(p) as f:
            rows = list(csv.reader(f))
        assert rows[0] == ["kernel_name", "avg_time", "TFLOPS", "speedup"]
        assert len(rows) == 1 + n_rows
        assert all(float(r[1]) > 0 and float(r[2]) > 0 for r in rows[1:])


def test_cli_check_mixed_qconfig_with_exporter_tile_config(out_dir):
    tc = out_dir / "tile_cfg.json"
    tc.write_text(json.dumps(json.load(open(GOLD / "tile_repr_golden.json"))["tile_cfg_file"]))
    res = run_mxmoe_gg.main(["--bs", "512", "--layer", "11", "--qconfig", str(LP1), "--tile_config", str(tc),
                             "--mode", "check", "--iters", "3"])
    assert res["qcfg_list"] == ["w4a4_g-1_sym", "w8a8_g-1_sym"]
    (v,) = res["variants"][11]
    assert all(nat.variant_supports(v, q) for q in res["qcfg_list"])
    _csv_ok(res["csv"], 2)  # torch.matmul baseline + the selected variant
    assert (out_dir / "out" / "workloads" / "qwen2_moe-wiki2-512-5.0_lp1.json").exists()


@pytest.mark.parametrize("qstr", ["w4a16_g128_asym", "w4a4_g128_sym", "w8a16_g-1_sym", "w8a8_g-1_sym_E4M3", "bf16",
                                  "fp16_accfp16"])
def test_cli_check_qstr(out_dir, qstr):
    res = run_mxmoe_gg.main(["--bs", "512", "--layer", "11", "--qstr", qstr, "--mode", "check", "--iters", "3"])
    vs = res["variants"][11]
    assert vs and all(nat.variant_supports(v, qstr) for v in vs)
    _csv_ok(res["csv"], 1 + len(vs))


def test_cli_tile_config_weight_only_maps_to_a_weight_only_variant(out_dir):
    tc = out_dir / "tile_cfg.json"
    tc.write_text(json.dumps({"11": "(TileConfig(BM=128, BN=128, BK=64, WM=2, WN=2, WK=1, STAGE=4, SPLITK=1, "
                                    "MMA='m16n8k16'),)"}))
    res = run_mxmoe_gg.main(["--bs", "512", "--layer", "11", "--qstr", "w4a16_g128_asym", "--tile_config", str(tc),
                             "--mode", "check", "--iters", "3", "--no-baseline"])
    (v,) = res["variants"][11]
    assert nat.variant_supports(v, "w4a16_g128_asym")
    _csv_ok(res["csv"], 1)
