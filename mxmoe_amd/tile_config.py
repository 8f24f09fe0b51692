"""tile_config JSON surface and the MI355X variant table.

Reference (SeaCatComplexes/MxMoE, mxmoe/kernels/tile_config.py): SUPPORTED_QCFG (:40-59),
get_info_from_qcfg_str (:288-294), TileConfig (:195-286) incl. smem sizing (:266-286), the
per-arch candidate lists (:330-610); compose_kernel.py:69-71 fusion rule (equal #warps).

The tile_config files written by bits_solver.export_qconfig (bits_solver.py:30, 67-68) hold
``{"<layer>": "(TileConfig(BM=..., ...), ...)"}`` — a Python repr, one TileConfig per strategy in
sorted-qcfg order. run_mxmoe_gg.py:102-107 passes that raw dict to TemplateGenerator, which expects
``{qcfg: [TileConfig]}`` (compose_kernel.py:88-91); both forms are accepted here. Reprs are parsed
with a restricted regex (never eval). A reference tile names an sm80/sm89 CUDA tile; it is mapped to
the nearest compiled MI355X variant (logged), because the HIP kernels are a fixed compiled table.
"""
from __future__ import annotations

import dataclasses
import json
import logging
import re
from typing import Optional, Union

log = logging.getLogger("mxmoe_amd.tile_config")

SUPPORTED_QCFG = [
    "fp16", "fp16_accfp16", "bf16",
    "w8a8_g-1_sym", "w8a8_g-1_sym_E4M3",
    "w4a4_g-1_sym", "w4a4_g128_sym",
    *[f"w{wbits}a16_g{gsize}_{sym}{ty}" for wbits in [8, 4, 2] for gsize in [-1, 128] for sym in ["sym", "asym"]
      for ty in ["", "_accfp16", "_bf16"]],
]

# what the MI355X kernels implement; the _accfp16 forms run as their f32-accumulating base type
# (MFMA has no fp16 accumulator); the weight-only _bf16 forms are not built
MI355X_QCFG = ["fp16", "fp16_accfp16", "bf16", "w8a8_g-1_sym", "w8a8_g-1_sym_E4M3", "w4a4_g-1_sym", "w4a4_g128_sym",
               *[f"w{w}a16_g{g}_{s}{t}" for w in (4, 8, 2) for g in (-1, 128) for s in ("sym", "asym")
                 for t in ("", "_accfp16")]]


def get_info_from_qcfg_str(qcfg: str) -> tuple[int, int, int, bool]:
    """(w_bits, a_bits, gsize, sym) from "w8a8_g-1_sym" (tile_config.py:288-294); format suffixes
    (``_E4M3``, ``_accfp16``, ``_bf16``) do not change the bit widths."""
    if qcfg in ("fp16", "fp16_accfp16", "bf16"):
        return 16, 16, -1, True
    splits = qcfg.split("_")
    wbits = int(splits[0].split("a")[0].split("w")[1])
    abits = int(splits[0].split("a")[1])
    gsize = int(splits[1].split("g")[1])
    sym = splits[2] == "sym"
    return wbits, abits, gsize, sym


@dataclasses.dataclass(frozen=True)
class TileConfig:
    BM: int = 64
    BN: int = 64
    BK: int = 64
    WM: int = 2
    WN: int = 2
    WK: int = 1
    STAGE: int = 2
    SPLITK: int = -1
    MMA: str = "MMA_FP16_FP32"

    @property
    def num_warps(self) -> int:
        return self.WM * self.WN * self.WK

    def smem_bytes_tile(self, a_bits: int = 16, w_bits: int = 16) -> int:
        """tile_config.py:276-286 (acc bytes: int32/float = 4)."""
        return max(self.STAGE * self.BM * self.BK * a_bits // 8 + self.STAGE * self.BN * self.BK * w_bits // 8,
                   4 * (self.WK - 1) * self.BM * self.BN)

    def smem_bytes_scale(self, quant: bool) -> int:
        """tile_config.py:266-274 (per-channel sym: one fp16 scale per row of A and B)."""
        return 2 * (self.BM + self.BN) if quant else 0


_TILE_RE = re.compile(r"TileConfig\((?P<body>[^()]*(?:\([^()]*\)[^()]*)*)\)")
_FIELD_RE = re.compile(r"\b(BM|BN|BK|WM|WN|WK|STAGE|SPLITK)\s*=\s*(-?\d+)|\bMMA\s*=\s*'([A-Za-z0-9_]+)'")


def parse_tile_repr(text: str) -> list[TileConfig]:
    """All TileConfig(...) in a repr string, in order (restricted regex; nested QConfig(...) ignored)."""
    out = []
    for m in _TILE_RE.finditer(text):
        kw = {}
        for f in _FIELD_RE.finditer(m.group("body")):
            if f.group(1):
                kw[f.group(1)] = int(f.group(2))
            else:
                kw["MMA"] = f.group(3)
        out.append(TileConfig(**kw))
    return out


def parse_tile_config_json(data: Union[str, dict], qcfgs: list[str], layer: Optional[int] = None) -> dict:
    """-> {qcfg: [TileConfig, ...]} from either accepted tile_config form."""
    if isinstance(data, str):
        with open(data) as f:
            data = json.load(f)
    qcfgs = sorted(qcfgs)
    if data and all(isinstance(v, str) for v in data.values()):  # exporter form {"<layer>": "repr"}
        key = str(layer) if layer is not None and str(layer) in data else next(iter(data))
        tiles = parse_tile_repr(data[key])
        if len(tiles) != len(qcfgs):
            raise ValueError(f"tile_config for layer {key} has {len(tiles)} tiles for {len(qcfgs)} qcfgs")
        return {q: [t] for q, t in zip(qcfgs, tiles)}
    out = {}
    for q in qcfgs:
        lst = data[q]
        out[q] = [t if isinstance(t, TileConfig) else
                  (parse_tile_repr(t)[0] if isinstance(t, str) else TileConfig(**t)) for t in lst]
    return out


# ------------------------------------------------------------------ MI355X variants

_VAR_RE = re.compile(r"^(\d+)\s+(\S+)\s+(.*)$")
_VQ_RE = re.compile(r"(\S+)=TileConfig\(BM=(\d+), BN=(\d+), BK=(\d+), WM=(\d+), WN=(\d+), WK=(\d+), STAGE=(\d+)\)")


def mi355x_variants() -> list[dict]:
    """Compiled variants from the library: [{id, name, tiles: {qcfg: TileConfig}}]."""
    from . import _native

    out = []
    for ln in _native.list_variants():
        m = _VAR_RE.match(ln)
        if not m:
            continue
        tiles = {}
        for q in _VQ_RE.finditer(m.group(3)):
            bm, bn, bk, wm, wn, wk, st = map(int, q.groups()[1:])
            tiles[q.group(1)] = TileConfig(BM=bm, BN=bn, BK=bk, WM=wm, WN=wn, WK=wk, STAGE=st)
        if m.group(2).startswith("abl_"):
            continue  # timing ablations compute wrong results by design
        out.append({"id": int(m.group(1)), "name": m.group(2), "tiles": tiles})
    return out


def variant_key(qcfg: str) -> str:
    """The key a variant lists a qcfg under: weight-only strategies by their base name
    (``w4a16_g128_asym`` -> ``w4a16``: one tile body serves every group size / symmetry);
    wxax and fp16 strategies by their full name (``w4a4_g128_sym`` is its own body)."""
    if qcfg == "fp16_accfp16":
        return "fp16"
    m = re.match(r"^(w\d+a16)_g-?\d+_a?sym(_accfp16)?$", qcfg)
    return m.group(1) if m else qcfg


def select_variant(tile_cfgs: Optional[dict] = None, default: int = 0, variants: Optional[list] = None) -> int:
    """Nearest compiled variant to the requested per-qcfg tiles (log-area + aspect distance).

    A variant with no tile body for one of the requested qcfgs is never chosen (infinite distance);
    if no variant covers all of them, ``default`` is returned."""
    if not tile_cfgs:
        return default
    import math

    best, best_d = default, float("inf")
    for v in (mi355x_variants() if variants is None else variants):
        d = 0.0
        for q, lst in tile_cfgs.items():
            have = v["tiles"].get(variant_key(q))
            if have is None:
                d = float("inf")
                break
            if lst:
                want = lst[0]
                d += abs(math.log2(want.BM / have.BM)) + abs(math.log2(want.BN / have.BN))
        if d < best_d:
            best, best_d = v["id"], d
    log.warning("tile_config mapped to MI355X variant %d (reference tiles are sm80/sm89 CUDA tiles)", best)
    return best
