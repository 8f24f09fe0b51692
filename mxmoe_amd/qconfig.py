"""qconfig JSON surface — mirrors mxmoe/kernels/qconfig.py and the exporter in bits_solver.py.

File format (bits_solver.py:25-71, export_qconfig):
  {"<layer>": {"experts": {"<e>": {"gate"|"up"|"down": QLinearConfig.to_dict()}}}, "LT": {...}}
QLinearConfig fields (qconfig.py:5-33): w_bits, w_gsize, w_sym, w_clip, a_bits, a_gsize, a_sym, a_clip.
``get_qcfg_list`` follows run_mxmoe_gg.py:11-29: the set of "w{w}a{a}_g{gsize}_{sym}" strings.
"""
from __future__ import annotations

import dataclasses
import json
from pathlib import Path
from typing import Union


@dataclasses.dataclass
class QLinearConfig:
    w_bits: int = 16
    w_gsize: int = -1
    w_sym: bool = False
    w_clip: tuple = (1.0, 1.0)
    a_bits: int = 16
    a_gsize: int = -1
    a_sym: bool = True
    a_clip: tuple = (1.0, 1.0)

    def __str__(self) -> str:
        return f"W{self.w_bits}A{self.a_bits}_g{self.w_gsize}_{'sym' if self.w_sym else 'asym'}"

    def to_dict(self) -> dict:
        return dataclasses.asdict(self)

    @property
    def qcfg(self) -> str:
        return f"w{self.w_bits}a{self.a_bits}_g{self.w_gsize}_{'sym' if self.w_sym else 'asym'}"

    @staticmethod
    def from_dict(d: dict) -> "QLinearConfig":
        return QLinearConfig(w_bits=d["w_bits"], w_gsize=d["w_gsize"], w_sym=d["w_sym"],
                             w_clip=tuple(d.get("w_clip", (1.0, 1.0))), a_bits=d["a_bits"],
                             a_gsize=d.get("a_gsize", -1), a_sym=d.get("a_sym", True),
                             a_clip=tuple(d.get("a_clip", (1.0, 1.0))))

    @staticmethod
    def from_qcfg(qname: str) -> "QLinearConfig":
        """bits_solver.py:32-37 parse_str."""
        parts = qname.split("_")
        w_bits, a_bits = [int(x) for x in parts[0].split("w")[1].split("a")]
        gsize = int(parts[1][1:])
        sym = parts[2] == "sym"
        return QLinearConfig(w_bits=w_bits, w_gsize=gsize, w_sym=sym, a_bits=a_bits, a_gsize=gsize, a_sym=sym)


def load_qconfig(path: Union[str, Path]) -> dict:
    with open(path) as f:
        return json.load(f)


def get_qcfg_list(qcfg: Union[str, Path, dict], target_layer: int) -> set:
    """Set of qcfg strings used by the target layer (run_mxmoe_gg.py:11-29); -1 = all layers."""
    if not isinstance(qcfg, dict):
        qcfg = load_qconfig(qcfg)
    qcfg = {k: v for k, v in qcfg.items() if k != "LT"}
    out = set()
    for layer_idx, v in qcfg.items():
        if target_layer != -1 and int(layer_idx) != target_layer:
            continue
        for _, qexp in v["experts"].items():
            for _, ql in qexp.items():
                out.add(f"w{ql['w_bits']}a{ql['a_bits']}_g{ql['w_gsize']}_{'sym' if ql['w_sym'] else 'asym'}")
    return out


def export_qconfig(strategies: dict, lt: dict | None = None) -> dict:
    """{layer: {expert: {weight_idx: qcfg_str}}} -> qconfig JSON dict (bits_solver.py:25-71)."""
    names = {0: "gate", 1: "up", 2: "down"}
    out = {
        str(layer): {"experts": {str(e): {names[int(w)]: QLinearConfig.from_qcfg(q).to_dict()
                                          for w, q in ecfg.items()} for e, ecfg in lcfg.items()}}
        for layer, lcfg in strategies.items()
    }
    if lt is not None:
        out["LT"] = lt
    return out


def uniform_qconfig(qcfg: str, num_layers: int, num_experts: int) -> dict:
    """Every linear of every expert with one qcfg (qconfig.py:83-97 build_uni_qmodel_cfg)."""
    return export_qconfig({layer: {e: {0: qcfg, 1: qcfg, 2: qcfg} for e in range(num_experts)}
                           for layer in range(num_layers)})
