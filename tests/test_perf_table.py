"""MI355X performance table: schema of the reference's
perf/performance_table.json (read by bits_solver.py:518-542, 647-653) and its cost function."""
from __future__ import annotations

import dataclasses
import json
from pathlib import Path

import pytest

from mxmoe_amd import perf_table as pt
from mxmoe_amd.tile_config import MI355X_QCFG, TileConfig

ROOT = Path(__file__).resolve().parent.parent
TABLE = ROOT / "mxmoe_amd" / "workloads" / "performance_table_mi355x.json"

# keys of the reference's perf/performance_table.json (data, copied as fixtures)
REF_KEY_W8A8 = ("TileConfig(BM=128, BN=128, BK=128, WM=2, WN=2, WK=1, STAGE=3, SPLITK=-1, MMA='MMA_S8_K32', "
                "QCFGA=QConfig(T_PACK='half', QBITS=8, GSIZE=-1, SYM=True, PACK_DIM='PackDim::K', USE_FP=False, "
                "T_SCALE='half'), QCFGB=QConfig(T_PACK='half', QBITS=8, GSIZE=-1, SYM=True, PACK_DIM='PackDim::K', "
                "USE_FP=False, T_SCALE='half'))")
REF_KEY_W4A16 = ("TileConfig(BM=64, BN=128, BK=128, WM=2, WN=2, WK=2, STAGE=4, SPLITK=-1, MMA='MMA_FP16_FP32', "
                 "QCFGA=NO_QUANT(T_PACK='half', QBITS=16, GSIZE=-1, SYM=True, PACK_DIM='PackDim::K', USE_FP=False, "
                 "T_SCALE='half'), QCFGB=QConfig(T_PACK='half', QBITS=4, GSIZE=128, SYM=False, "
                 "PACK_DIM='PackDim::MN', USE_FP=False, T_SCALE='half'))")


def test_tile_repr_matches_reference_keys():
    assert pt.tile_repr(TileConfig(128, 128, 128, 2, 2, 1, 3, -1, "MMA_S8_K32"), "w8a8_g-1_sym") == REF_KEY_W8A8
    assert pt.tile_repr(TileConfig(64, 128, 128, 2, 2, 2, 4, -1, "MMA_FP16_FP32"), "w4a16_g128_asym") == REF_KEY_W4A16


def test_fit_line_recovers_slope():
    xs = [256, 512, 1024, 2048]
    a, b, se = pt.fit_line(xs, [0.01 + 2e-4 * x for x in xs])
    assert abs(a - 0.01) < 1e-12 and abs(b - 2e-4) < 1e-15 and se < 1e-12


@dataclasses.dataclass
class _P:
    M: int
    N: int
    K: int


def test_runtime_cost_is_inc_times_tiles():
    t = TileConfig(256, 256, 256, 2, 4, 1, 2, -1, "MFMA_I8_K64")
    table = {q: {str(k): {pt.tile_repr(t, q): {"inc": 0.001 * k, "first_iter_cost": 0.0, "stderr": 0.0}}
                 for k in pt.K_CLASSES} for q in ("w8a8_g-1_sym", "w4a4_g-1_sym")}
    tiles = {q: t for q in table}
    cost = pt.runtime_cost([[_P(300, 2816, 2048), _P(8192, 2048, 1408)]], ["w8a8_g-1_sym", "w4a4_g-1_sym"], table, tiles)
    assert cost[0][0] == [pytest.approx(0.002 * 2 * 11)] * 2  # K=2048 -> key "2"; 2 x 11 tiles
    assert cost[0][1][0] == pytest.approx(0.001 * 1408 / 1024 * 32 * 8)  # K=1408 -> key "1", scaled by K
    assert pt.tiles_from_table(table)["w8a8_g-1_sym"] == dataclasses.replace(t, MMA="MFMA_I8_K64")


@pytest.mark.skipif(not TABLE.exists(), reason="table not measured yet")
def test_committed_table_has_reference_schema():
    table = json.loads(TABLE.read_text())
    assert set(table) == set(MI355X_QCFG)
    for q, per_k in table.items():
        assert set(per_k) == {str(k) for k in pt.K_CLASSES}  # bits_solver reads "1" and "3"
        for k, entries in per_k.items():
            (rep, e), = entries.items()
            assert rep.startswith("TileConfig(") and "QCFGA=" in rep
            assert e["inc"] > 0 and "first_iter_cost" in e and "stderr" in e
