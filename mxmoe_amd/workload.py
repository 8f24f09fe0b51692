"""Workload JSON surface (problem lists per layer) — mirrors mxmoe/kernels/gen_workload.py.

Reference behaviour kept (SeaCatComplexes/MxMoE, gen_workload.py):
  * MODEL_ID_TO_LAYERS ............................................. :16-21
  * qstr -> {w_bits, a_bits, gsize, sym} parsing .................... :51-57
  * per routed expert e: gate_up [int(p_e*T*topk), 2N, K], down [int(p_e*T*topk), K, N] .. :93-96
  * shared expert appended last: gate_up [T, 2N*S, K], down [T, K, N*S] (S may be a float) .. :99-101
  * the shared expert's down projection takes the "gate" qcfg (reference behaviour, :101) — kept
    by default so generated workloads match the reference byte for byte (``shared_down_qcfg``)
  * output JSON {"num_tokens": T, "layer-L": {"gate_up": [...], "down": [...]}} .... :68-106
The workload JSON is read like test.cu's parse_json_input (test.cu:652-674): floats -> int.
"""
from __future__ import annotations

import dataclasses
import json
import os
from pathlib import Path
from typing import Literal, Optional

import numpy as np

from .qconfig import load_qconfig

WORKLOAD_DIR = Path(__file__).resolve().parent / "workloads"

MODEL_ID_TO_LAYERS = {
    "qwen2_moe": 24,
    "qwen2_moe_57b": 28,
    "ds2": 27,
    "mixtral": 32,
}

# MoE geometry per model (moe_tracer.py:42-56; public model configs): hidden K, expert intermediate N,
# routed experts, top-k, shared experts (as the multiplier S used by gen_workload.py:99-101).
MODEL_SHAPES = {
    "qwen2_moe": dict(K=2048, N=1408, E=60, topk=4, S=4.0),
    "ds2": dict(K=2048, N=1408, E=64, topk=6, S=2),
    "qwen2_moe_57b": dict(K=3584, N=2560, E=64, topk=8, S=8.0),
    "mixtral": dict(K=4096, N=14336, E=8, topk=2, S=0),
}


@dataclasses.dataclass
class QShape:
    """One problem of a workload (test.cu:63-87)."""

    shape: list
    w_bits: int = 16
    a_bits: int = 16
    gsize: int = -1
    sym: bool = True
    fmt: str = ""  # "" | "E4M3" | "bf16" (written to JSON only when set: reference files are unchanged)

    @property
    def M(self) -> int:
        return int(self.shape[0])

    @property
    def N(self) -> int:
        return int(self.shape[1])

    @property
    def K(self) -> int:
        return int(self.shape[2])

    @property
    def qcfg(self) -> str:
        if self.w_bits == 16 and self.a_bits == 16:
            return "bf16" if self.fmt == "bf16" else "fp16"
        return f"w{self.w_bits}a{self.a_bits}_g{self.gsize}_{'sym' if self.sym else 'asym'}" + \
            ("_E4M3" if self.fmt == "E4M3" else "")

    @property
    def flops(self) -> int:
        return 2 * self.M * self.N * self.K

    def to_json(self) -> dict:
        d = {"shape": list(self.shape), "w_bits": self.w_bits, "a_bits": self.a_bits, "gsize": self.gsize,
             "sym": self.sym}
        if self.fmt:
            d["fmt"] = self.fmt
        return d

    @staticmethod
    def from_json(j: dict) -> "QShape":
        return QShape(shape=[int(x) for x in j["shape"]], w_bits=int(j["w_bits"]), a_bits=int(j["a_bits"]),
                      gsize=int(j["gsize"]), sym=bool(j["sym"]), fmt=str(j.get("fmt", "")))


def parse_qstr(qstr: str) -> dict:
    """gen_workload.py:51-57; also the SUPPORTED_QCFG forms that reference parser cannot read
    (``bf16``, ``fp16[_accfp16]``, ``..._E4M3``; ``_accfp16`` runs as its f32-accumulating base)."""
    if qstr in ("fp16", "fp16_accfp16", "bf16"):
        d = dict(FP16_QCFG)
        if qstr == "bf16":
            d["fmt"] = "bf16"
        return d
    d = {
        "w_bits": int(qstr.split("w")[1].split("a")[0]),
        "a_bits": int(qstr.split("a")[1].split("_g")[0]),
        "gsize": int(qstr.split("_g")[1].split("_")[0]),
        "sym": "asym" not in qstr,
    }
    if qstr.endswith("_E4M3"):
        d["fmt"] = "E4M3"
    return d


FP16_QCFG = {"w_bits": 16, "a_bits": 16, "gsize": -1, "sym": True}


def freq_to_prob(freq: list) -> list:
    total = sum(freq)
    return [f / total for f in freq]


def generate_workload_from_trace(trace: dict, num_total_tokens: int, layer_id: int = -1,
                                 qconfig: Optional[dict] = None, qstr: Optional[str] = None,
                                 shared_down_qcfg: Literal["gate", "down"] = "gate") -> dict:
    """Problem lists for every (or one) layer of a gate trace (gen_workload.py:38-110)."""
    if qconfig is not None and qstr is not None:
        raise ValueError("qconfig and qstr are exclusive")
    if qconfig is not None:
        qconfig = {k: v for k, v in qconfig.items() if k != "LT"}
        uni = None
    else:
        uni = parse_qstr(qstr) if qstr is not None else dict(FP16_QCFG)

    topk = trace["topk"]
    N, K = trace["NK"]
    S = trace["num_shared_experts"]
    result: dict = {"num_tokens": num_total_tokens}
    for key, value in trace.items():
        if not key.startswith("layer-"):
            continue
        layer_idx = key.split("-")[1]
        if layer_id != -1 and layer_idx != str(layer_id):
            continue

        def lin(exp_idx: str, linear: str) -> dict:
            if uni is not None:
                return dict(uni)
            c = qconfig[layer_idx]["experts"][exp_idx][linear]
            return {"w_bits": c["w_bits"], "a_bits": c["a_bits"], "gsize": c["w_gsize"], "sym": c["w_sym"]}

        prob = freq_to_prob(value["access_freq"])
        E = len(prob)
        shapes: dict = {"gate_up": [], "down": []}
        for e, p in enumerate(prob):
            m = int(p * num_total_tokens * topk)
            shapes["gate_up"].append({"shape": [m, N * 2, K], **lin(str(e), "gate")})
            shapes["down"].append({"shape": [m, K, N], **lin(str(e), "down")})
        if S != 0:
            shapes["gate_up"].append({"shape": [int(num_total_tokens), N * 2 * S, K], **lin(str(E), "gate")})
            shapes["down"].append({"shape": [int(num_total_tokens), K, N * S], **lin(str(E), shared_down_qcfg)})
        result[f"layer-{layer_idx}"] = shapes
    return result


def save_workload(wl: dict, path: str) -> None:
    os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
    with open(path, "w") as f:
        json.dump(wl, f, indent=2)


def load_workload(path_or_dict) -> dict[str, dict[str, list[QShape]]]:
    """Parse a workload JSON (test.cu:652-674): {layer: {gate_up|down: [QShape]}}; num_tokens skipped."""
    if isinstance(path_or_dict, dict):
        d = path_or_dict
    else:
        with open(path_or_dict) as f:
            d = json.load(f)
    out = {}
    for k, v in d.items():
        if k == "num_tokens":
            continue
        out[k] = {gg: [QShape.from_json(p) for p in lst] for gg, lst in v.items()}
    return out


# ---------------------------------------------------------------- synthetic workloads (bench)

def qwen2_hist() -> dict:
    with open(WORKLOAD_DIR / "qwen2_moe_hist_bs8192.json") as f:
        return json.load(f)


def qwen2_layer11_trace(bs_ref: int = 8192) -> dict:
    """A gate trace whose layer-11 access frequencies are the committed bs=8192 histogram (§8d)."""
    h = qwen2_hist()
    return {"topk": h["topk"], "NK": [h["moe_intermediate"], h["hidden"]], "num_shared_experts": h["num_shared_experts"],
            "layer-11": {"access_freq": h["M"]}}


def qwen2_layer11_workload(bs: int = 8192, qconfig: Optional[dict] = None, qstr: Optional[str] = None) -> dict:
    """qwen2_moe 'layer-11' problems. At bs=8192 the routed M_e are exactly the committed histogram."""
    h = qwen2_hist()
    if bs == h["num_tokens"]:
        wl = generate_workload_from_trace(qwen2_layer11_trace(), bs, 11, qconfig=qconfig, qstr=qstr)
        for gg in ("gate_up", "down"):  # int(p*T*topk) truncation differs by <=1 row: pin the committed M_e
            for p, m in zip(wl["layer-11"][gg][:-1], h["M"]):
                p["shape"][0] = m
        return wl
    return generate_workload_from_trace(qwen2_layer11_trace(), bs, 11, qconfig=qconfig, qstr=qstr)


def synthetic_trace(model: str, bs: int = 8192, seed: int = 0, layer: int = 1) -> dict:
    """Seeded routing for a model the reference ships no gate trace for (only qwen2_moe's histogram is
    in the tree): M_e ~ multinomial(bs*topk, dirichlet(20*1_E)), the model's MoE
    geometry from MODEL_SHAPES (gen_workload.py:16-21 model ids; moe_tracer.py:42-56)."""
    s = MODEL_SHAPES[model]
    rng = np.random.default_rng(seed)
    p = rng.dirichlet(20.0 * np.ones(s["E"]))
    m = rng.multinomial(bs * s["topk"], p)
    return {"topk": s["topk"], "NK": [s["N"], s["K"]], "num_shared_experts": s["S"],
            f"layer-{layer}": {"access_freq": [int(x) for x in m]}}


def ds2_trace(bs: int = 8192, seed: int = 0) -> dict:
    """DeepSeek-V2-Lite routing: M_e ~ multinomial(bs*6, dirichlet(20*1_64))."""
    return synthetic_trace("ds2", bs, seed, layer=1)


def model_workload(model: str, bs: int = 8192, qconfig: Optional[dict] = None, qstr: Optional[str] = None,
                   seed: int = 0) -> dict:
    """One layer ("layer-1") of a model with seeded synthetic routing (mixtral, qwen2_moe_57b, ds2)."""
    return generate_workload_from_trace(synthetic_trace(model, bs, seed, layer=1), bs, 1, qconfig=qconfig, qstr=qstr)


def ds2_workload(bs: int = 8192, qconfig: Optional[dict] = None, qstr: Optional[str] = None, seed: int = 0) -> dict:
    return generate_workload_from_trace(ds2_trace(bs, seed), bs, 1, qconfig=qconfig, qstr=qstr)


def ds2_mixed_qconfig(seed: int = 0, frac: float = 0.25, layer: int = 1) -> dict:
    """DeepSeek-V2-Lite mixed w4a4 + w8a8 allocation (the reference ships no qconfig
    for this model): a seeded (PCG64) random order of (expert, gate_up | down) blocks is scanned
    greedily, each block turned w8a8 while the w8a8 weight units stay <= frac of all units; units per
    linear are 1 (routed) or 2 (shared expert, index E), gate and up tied. Export format of
    bits_solver.py:25-71. Pinned by tests/golden/ds2_mixed_alloc.json."""
    E = MODEL_SHAPES["ds2"]["E"]
    blocks = [(e, lin) for e in range(E + 1) for lin in ("gate_up", "down")]

    def units(e: int, lin: str) -> int:
        return (2 if e == E else 1) * (2 if lin == "gate_up" else 1)

    budget = frac * sum(units(*b) for b in blocks)
    w8, used = set(), 0
    for i in np.random.default_rng(seed).permutation(len(blocks)):
        b = blocks[int(i)]
        if used + units(*b) <= budget:
            w8.add(b)
            used += units(*b)

    def cfg(bits: int) -> dict:
        return {"w_bits": bits, "w_gsize": -1, "w_sym": True, "w_clip": [1.0, 1.0],
                "a_bits": bits, "a_gsize": -1, "a_sym": True, "a_clip": [1.0, 1.0]}

    experts = {}
    for e in range(E + 1):
        gu, dn = (8 if (e, "gate_up") in w8 else 4), (8 if (e, "down") in w8 else 4)
        experts[str(e)] = {"gate": cfg(gu), "up": cfg(gu), "down": cfg(dn)}
    return {str(layer): {"experts": experts}}


def w4a16_w8a8_qconfig(seed: int = 0, frac: float = 1.0 / 16, layer: int = 11) -> dict:
    """qwen2_moe small-batch mixed scheme: w4a16_g-1_asym + w8a8_g-1_sym per linear block, the pairing
    the reference hand-instantiates as one fused kernel (hz_fused.cuh:14-125, QConfig<half, false, 4,
    -1, ...> + QCFG_W8A8; mxmoe_w4a16_w8a8_bs256 at ref_bind.cu:412). frac = 1/16 of the weight units
    w8a8 gives the reference's published "W4.25A15.5" average (8/16 + 4 * 15/16 = 4.25 weight bits,
    8/16 + 16 * 15/16 = 15.5 activation bits). Same seeded greedy scan as
    ds2_mixed_qconfig; the shared expert (index E, 4x the intermediate width) weighs 4 units."""
    E = MODEL_SHAPES["qwen2_moe"]["E"]
    blocks = [(e, lin) for e in range(E + 1) for lin in ("gate_up", "down")]

    def units(e: int, lin: str) -> int:
        return (4 if e == E else 1) * (2 if lin == "gate_up" else 1)

    budget = frac * sum(units(*b) for b in blocks)
    w8, used = set(), 0
    for i in np.random.default_rng(seed).permutation(len(blocks)):
        b = blocks[int(i)]
        if used + units(*b) <= budget:
            w8.add(b)
            used += units(*b)
    w4a16 = {"w_bits": 4, "w_gsize": -1, "w_sym": False, "w_clip": [1.0, 1.0],
             "a_bits": 16, "a_gsize": -1, "a_sym": True, "a_clip": [1.0, 1.0]}
    w8a8 = {"w_bits": 8, "w_gsize": -1, "w_sym": True, "w_clip": [1.0, 1.0],
            "a_bits": 8, "a_gsize": -1, "a_sym": True, "a_clip": [1.0, 1.0]}
    experts = {}
    for e in range(E + 1):
        gu = w8a8 if (e, "gate_up") in w8 else w4a16
        dn = w8a8 if (e, "down") in w8 else w4a16
        experts[str(e)] = {"gate": dict(gu), "up": dict(gu), "down": dict(dn)}
    return {str(layer): {"experts": experts}}


def mixed_qconfig_lp1() -> dict:
    """The committed mixed w4a4+w8a8 (wbits 5.0) qconfig solved from the reference's bits_model-1.lp."""
    return load_qconfig(WORKLOAD_DIR / "qconfig_qwen2_moe_w4a4+w8a8_wbits5.0_lp1.json")


def layer_problems(wl: dict, layer: Optional[str] = None) -> dict[str, list[QShape]]:
    parsed = load_workload(wl)
    key = layer or next(iter(parsed))
    return parsed[key]
