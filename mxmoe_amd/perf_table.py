"""MI355X kernel performance table for the accuracy/performance co-design solver.

The reference's ILP (mxmoe/quant/bits_solver.py:518-542, get_runtime_cost) prices a problem under a
quantisation strategy as ``performance_table[qcfg][key][repr(tile)]["inc"] * num_tiles(tile)``
(``ProblemShape.num_tiles``, bits_solver.py:109-110), reading the table from
``perf/performance_table.json`` (bits_solver.py:647-653). That file holds sm89 numbers; this module
produces the same schema for the MI355X kernels and restates the cost function:

  {qcfg: {key: {"TileConfig(BM=..., ...)": {"first_iter_cost": ms, "inc": ms per tile, "stderr": ms}}}}

* ``qcfg``: every strategy the MI355X kernels implement (``tile_config.MI355X_QCFG``); the
  ``_accfp16`` strategies run their base type's kernel, so their entries are copies of the base
  entries (``ALIASES``, written by ``dump``), and only ``MEASURED_QCFG`` is swept.
* ``key``: the reference's generator is not in its tree and its key semantics are undocumented
  (bits_solver reads "1" for weight-only and "3" for weight-activation strategies). Here key k is
  the K class K = 1024·k (k = 1..4); every key is present for every qcfg, so the reference's
  lookups resolve.
* the tile: the tile the AUTO policy runs for that qcfg (``mxmoe_gg_list_variants``), in the
  reference TileConfig repr form.
* ``inc`` / ``first_iter_cost`` / ``stderr``: least-squares slope / intercept / slope standard error
  of one launch's device time (HIP events, median of repeats) against its tile count, over calls of
  P identical problems (4 x 4 tiles each) — the per-tile increment of a chip-filling call, i.e. what
  ``inc * num_tiles`` needs to estimate a layer's time.
"""
from __future__ import annotations

import dataclasses
import json
import math
from typing import Optional, Sequence

from .tile_config import MI355X_QCFG, TileConfig, get_info_from_qcfg_str

K_CLASSES = (1, 2, 3, 4)  # key k <-> K = 1024 * k
ALIASES = {q: q.replace("_accfp16", "") for q in MI355X_QCFG if "_accfp16" in q}
MEASURED_QCFG = [q for q in MI355X_QCFG if q not in ALIASES]


def _fmt(qcfg: str) -> str:
    from .groupgemm import QParams

    return QParams.from_qcfg(qcfg).fmt


def tile_repr(t: TileConfig, qcfg: str) -> str:
    """The reference TileConfig repr (tile_config.py:195-264 dataclass repr, as in performance_table.json)."""
    w, a, g, sym = get_info_from_qcfg_str(qcfg)

    use_fp = qcfg.endswith("_E4M3")  # QCFG_W8A8_E4M3 (tile_config.py:192): USE_FP=True

    def qc(bits, gs, sy, dim="K"):
        kind = "NO_QUANT" if bits >= 16 else "QConfig"
        if bits >= 16:
            gs, sy, dim = -1, True, "K"
        return (f"{kind}(T_PACK='half', QBITS={bits}, GSIZE={gs}, SYM={sy}, PACK_DIM='PackDim::{dim}', "
                f"USE_FP={use_fp and bits < 16}, T_SCALE='half')")

    # weight-only B is packed along N (pack_weightonly, quantize.cuh:318-421): PackDim::MN
    return (f"TileConfig(BM={t.BM}, BN={t.BN}, BK={t.BK}, WM={t.WM}, WN={t.WN}, WK={t.WK}, STAGE={t.STAGE}, "
            f"SPLITK={t.SPLITK}, MMA='{t.MMA}', QCFGA={qc(a, g, sym)}, "
            f"QCFGB={qc(w, g, sym, 'MN' if a >= 16 else 'K')})")


def fit_line(xs: Sequence[float], ys: Sequence[float]) -> tuple[float, float, float]:
    """(intercept, slope, slope standard error) of an ordinary least-squares line."""
    n = len(xs)
    mx, my = sum(xs) / n, sum(ys) / n
    sxx = sum((x - mx) ** 2 for x in xs)
    sxy = sum((x - mx) * (y - my) for x, y in zip(xs, ys))
    b = sxy / sxx
    a = my - b * mx
    se = math.sqrt(sum((y - a - b * x) ** 2 for x, y in zip(xs, ys)) / (n - 2) / sxx) if n > 2 else 0.0
    return a, b, se


def num_tiles(M: int, N: int, tile: TileConfig) -> int:
    """bits_solver.py:109-110."""
    return ((M + tile.BM - 1) // tile.BM) * ((N + tile.BN - 1) // tile.BN)


def k_key(K: int) -> str:
    """The table key of a problem's K (nearest measured K class)."""
    return str(min(K_CLASSES, key=lambda c: abs(1024 * c - K)))


def runtime_cost(workloads, strategies: Sequence[str], table: dict, tiles: dict) -> list:
    """get_runtime_cost (bits_solver.py:518-542) on the MI355X table: cost[e][i][j] = inc * num_tiles
    of problem i of expert e under strategy j, with the inc of the nearest K class scaled by
    K / K_class (a tile's mainloop is linear in K; the reference reads one fixed key per strategy
    family, which misprices a K = 1408 down projection by 27 % against its 1024 class —
    tests/test_perf_table_gpu.py checks the prediction against measured layer calls). One compiled
    tile per strategy runs every strategy in one launch, so there is no fusion enumeration (the
    reference's outer tile-combination axis). ``workloads[e][i]`` has M, N, K; ``tiles[qcfg]`` is
    the TileConfig the table was measured with."""
    out = []
    for exp in workloads:
        row = []
        for w in exp:
            kk = k_key(w.K)
            scale = w.K / (1024 * int(kk))
            row.append([table[q][kk][tile_repr(tiles[q], q)]["inc"] * scale * num_tiles(w.M, w.N, tiles[q])
                        if q in table else
                        table[ALIASES[q]][kk][tile_repr(tiles[ALIASES[q]], ALIASES[q])]["inc"] * scale *
                        num_tiles(w.M, w.N, tiles[ALIASES[q]])
                        for q in strategies])
        out.append(row)
    return out


def tiles_from_table(table: dict) -> dict:
    """qcfg -> TileConfig recovered from the table's repr keys (restricted regex parser)."""
    from .tile_config import parse_tile_repr

    out = {}
    for q, per_k in table.items():
        rep = next(iter(next(iter(per_k.values())).keys()))
        out[q] = parse_tile_repr(rep)[0]
    return out


def auto_tiles(qcfgs: Sequence[str] = MI355X_QCFG) -> dict:
    """qcfg -> the TileConfig of the variant the library's AUTO policy runs for a call of that qcfg."""
    from . import _native as nat
    from .tile_config import mi355x_variants

    by_id = {v["id"]: v for v in mi355x_variants()}
    out = {}
    for q in qcfgs:
        w, a, g, sym = get_info_from_qcfg_str(q)
        vid = nat.default_variant()
        if q == "w4a4_g-1_sym":  # AUTO: int4-only calls run the 256x128 2-WG/CU kernel
            vid = next(v["id"] for v in by_id.values() if v["name"].startswith("v3_256x128"))
        tiles = by_id[vid]["tiles"]
        t = tiles[q if q in tiles else f"w{w}a16"]
        mma = ("MFMA_F8_K128" if q.endswith("_E4M3") else "MFMA_BF16_F32" if q == "bf16" else
               "MFMA_F16_F32" if a == 16 else "MFMA_I8_K64")
        out[q] = dataclasses.replace(t, MMA=mma)
    return out


def measure(qcfgs: Sequence[str] = MEASURED_QCFG, sizes: Sequence[int] = (16, 32, 64, 128, 256), iters: int = 20,
            device: Optional[str] = None, log=None) -> dict:
    """Run the sweep on the current GPU; returns the table (reference schema + the raw points)."""
    import torch

    from .groupgemm import GroupGemm
    from .harness import build_layer_inputs, time_launches
    from .workload import QShape

    tiles = auto_tiles(qcfgs)
    table: dict = {}
    for q in qcfgs:
        w, a, g, sym = get_info_from_qcfg_str(q)
        t = tiles[q]
        table[q] = {}
        for k in K_CLASSES:
            K = 1024 * k
            M, N = 4 * t.BM, 4 * t.BN  # 16 tiles per problem
            shapes = [QShape(shape=[M, N, K], w_bits=w, a_bits=a, gsize=g, sym=sym, fmt=_fmt(q))
                      for _ in range(max(sizes))]
            inp = build_layer_inputs(shapes, device=device or "cuda", seed=k)
            xs, ys = [], []
            for P in sizes:
                gg = GroupGemm(inp.problems[:P])
                ys.append(time_launches(gg.launch, warmup=3, iters=iters)["median_ms"])
                xs.append(gg.total_tiles)
                del gg
            a0, b, se = fit_line(xs, ys)
            table[q][str(k)] = {tile_repr(t, q): {"first_iter_cost": round(a0, 5), "inc": round(b, 7), "stderr": se,
                                                   "tiles": xs, "ms": [round(y, 5) for y in ys], "K": K}}
            if log:
                log(f"{q} K={K}: inc {b * 1e3:.3f} us/tile, first {a0:.4f} ms")
            del inp
            torch.cuda.empty_cache()
    return table


def with_aliases(table: dict) -> dict:
    """The table plus an entry for every ``_accfp16`` strategy whose base type was measured (the
    same kernel runs both), keyed by the alias's own TileConfig repr."""
    out = dict(table)
    tiles = tiles_from_table(table)
    for alias, base in ALIASES.items():
        if base in table:
            out[alias] = {k: {tile_repr(tiles[base], alias): e for e in v.values()} for k, v in table[base].items()}
    return out


def dump(table: dict, path: str, merge: bool = False) -> None:
    """Write the table (with alias entries); merge=True keeps the other qcfgs of an existing file."""
    import os

    if merge and os.path.exists(path):
        with open(path) as f:
            old = json.load(f)
        old.update(table)
        table = old
    table = with_aliases({q: v for q, v in table.items() if q not in ALIASES})
    with open(path, "w") as f:
        json.dump(table, f, indent=1)
