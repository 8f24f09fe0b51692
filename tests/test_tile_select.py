"""tile_config JSON -> compiled MI355X variant (tile_config.select_variant), with a mocked variant
list (CPU) and against the library's own listing (weight-only qcfgs were never matched,
so variant 0 — which has no weight-only body — was picked)."""
from __future__ import annotations

from mxmoe_amd.tile_config import TileConfig, parse_tile_config_json, select_variant, variant_key

T = lambda bm, bn: TileConfig(BM=bm, BN=bn, BK=64, WM=2, WN=4, WK=1, STAGE=2)  # noqa: E731
MOCK = [
    {"id": 0, "name": "v0", "tiles": {"fp16": T(128, 128), "w8a8_g-1_sym": T(128, 128), "w4a4_g-1_sym": T(128, 128)}},
    {"id": 3, "name": "v2", "tiles": {"fp16": T(256, 256), "w8a8_g-1_sym": T(256, 256), "w4a4_g-1_sym": T(256, 256),
                                      "w4a16": T(256, 256), "w8a16": T(256, 256), "w2a16": T(256, 256),
                                      "w4a4_g128_sym": T(256, 256)}},
    {"id": 7, "name": "v3", "tiles": {"fp16": T(256, 128), "w8a8_g-1_sym": T(256, 128), "w4a4_g-1_sym": T(256, 128)}},
]


def test_variant_key_normalises_weight_only():
    assert variant_key("w4a16_g128_asym") == "w4a16"
    assert variant_key("w8a16_g-1_sym") == "w8a16"
    assert variant_key("w2a16_g128_sym") == "w2a16"
    assert variant_key("w4a4_g128_sym") == "w4a4_g128_sym"
    assert variant_key("w8a8_g-1_sym") == "w8a8_g-1_sym"
    assert variant_key("fp16") == "fp16"


def test_select_nearest_among_covering_variants():
    assert select_variant({"w8a8_g-1_sym": [T(128, 128)]}, default=3, variants=MOCK) == 0
    assert select_variant({"w4a4_g-1_sym": [T(256, 128)]}, default=3, variants=MOCK) == 7
    assert select_variant({"fp16": [T(256, 256)], "w8a8_g-1_sym": [T(256, 256)]}, default=0, variants=MOCK) == 3


def test_select_never_picks_a_variant_without_the_body():
    # weight-only and g128 qcfgs exist only in v2: v0's closer tile shape must not win
    assert select_variant({"w4a16_g128_asym": [T(128, 128)]}, default=0, variants=MOCK) == 3
    assert select_variant({"w4a4_g128_sym": [T(128, 128)], "w8a8_g-1_sym": [T(128, 128)]}, default=0,
                          variants=MOCK) == 3
    # nothing covers an unknown qcfg: the default stands
    assert select_variant({"w3a3_g-1_sym": [T(128, 128)]}, default=7, variants=MOCK) == 7


def test_exporter_form_maps_through():
    tiles = parse_tile_config_json({"11": "(TileConfig(BM=128, BN=128, BK=64, WM=2, WN=2, WK=1, STAGE=4, SPLITK=1, "
                                          "MMA='m16n8k16'),)"}, ["w4a16_g128_asym"], layer=11)
    assert select_variant(tiles, default=0, variants=MOCK) == 3
