"""One qwen2_moe layer-11 MoE FFN step at bs=8192 (LP-1 mixed w4a4 + w8a8 qconfig, routed histogram of
the committed workload, random weights) on the device: quant_act -> gate_up GroupGEMM -> SiLU·mul +
quant -> down GroupGEMM -> combine, with the GroupGEMMs planned once, timed per stage and as a
whole, unfused (silu_mul_quant) against the fused SiLU epilogue (MXMOE_GG_EPI_SILU_MUL +
quant_slots). Alternating rounds; the two layers' outputs are checked bit-identical first.

python tools/moe_layer_bench.py [--rounds 4] [--iters 30] > gpurun_out/moe_layer.jsonl
"""
from __future__ import annotations

import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from mxmoe_amd import moe  # noqa: E402
from mxmoe_amd.groupgemm import GroupGemm, Problem, QParams  # noqa: E402
from mxmoe_amd.harness import time_launches  # noqa: E402
from mxmoe_amd.workload import load_workload, mixed_qconfig_lp1, qwen2_layer11_workload  # noqa: E402

T, TOPK, E, H, N, NS = 8192, 4, 60, 2048, 1408, 5632


class Step:
    """A MoEFFN forward with every launch planned once (the plumbing kernels relaunch on the same
    buffers; both GroupGEMMs keep their plans)."""

    def __init__(self, layer: moe.MoEFFN, hidden, ids, wts):
        dev = hidden.device
        self.r = r = moe.route(ids, layer.E)
        self.a1 = moe.quant_act(hidden, r, layer.tag1, layer.has_shared)
        f = 1 if layer.fuse_silu else 2
        self.h1 = torch.empty(T * TOPK, f * layer.N, dtype=torch.float16, device=dev)
        self.h1s = torch.empty(T, f * layer.Ns, dtype=torch.float16, device=dev)
        p1 = []
        for e, s in enumerate(self.a1.segs):
            if s.rows:
                w = layer.w1[e]
                C = self.h1s if e == layer.E else self.h1[s.first_slot:s.first_slot + s.rows]
                p1.append(Problem(A=self.a1.A(e), B=w.B, C=C, M=s.rows, N=w.N, K=w.K, q=w.q, scale_a=self.a1.scale(e),
                                  scale_b=w.scale_b, silu=layer.fuse_silu))
        self.g1 = GroupGemm(p1)
        self.a2 = moe.silu_mul_quant(self.h1, self.h1s, r, layer.tag2, activated=layer.fuse_silu)
        self.y = torch.empty(T * TOPK, H, dtype=torch.float16, device=dev)
        self.ys = torch.empty(T, H, dtype=torch.float16, device=dev)
        p2 = []
        for e, s in enumerate(self.a2.segs):
            if s.rows:
                w = layer.w2[e]
                C = self.ys if e == layer.E else self.y[s.first_slot:s.first_slot + s.rows]
                p2.append(Problem(A=self.a2.A(e), B=w.B, C=C, M=s.rows, N=w.N, K=w.K, q=w.q, scale_a=self.a2.scale(e),
                                  scale_b=w.scale_b))
        self.g2 = GroupGemm(p2)
        self.out = torch.empty(T, H, dtype=torch.float16, device=dev)
        self.w = wts.to(torch.float32).contiguous()
        self.stages = {"quant_act": self.a1.relaunch, "gate_up": self.g1.launch, "act_quant": self.a2.relaunch,
                       "down": self.g2.launch, "combine": self.combine}

    def combine(self):
        moe.combine_into(self.out, self.y, self.r.inv_slot, self.w, self.ys, TOPK)

    def __call__(self):
        for fn in self.stages.values():
            fn()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=4)
    ap.add_argument("--iters", type=int, default=30)
    args = ap.parse_args()
    dev = "cuda"
    layer = load_workload(qwen2_layer11_workload(T, qconfig=mixed_qconfig_lp1()))["layer-11"]
    qcfg = [(QParams(a.a_bits, a.w_bits, a.gsize, a.sym), QParams(b.a_bits, b.w_bits, b.gsize, b.sym))
            for a, b in zip(layer["gate_up"], layer["down"])]
    counts = [s.M for s in layer["gate_up"][:E]]
    counts[0] += T * TOPK - sum(counts)
    g = torch.Generator().manual_seed(0)
    ids = torch.repeat_interleave(torch.arange(E, dtype=torch.int32), torch.tensor(counts))
    ids = ids[torch.randperm(ids.numel(), generator=g)].view(T, TOPK).contiguous().to(dev)
    gate_up = [((torch.rand(2 * N, H, generator=g) * 2 - 1) * 0.05).half().to(dev) for _ in range(E)]
    gate_up.append(((torch.rand(2 * NS, H, generator=g) * 2 - 1) * 0.05).half().to(dev))
    down = [((torch.rand(H, N, generator=g) * 2 - 1) * 0.05).half().to(dev) for _ in range(E)]
    down.append(((torch.rand(H, NS, generator=g) * 2 - 1) * 0.05).half().to(dev))
    hidden = ((torch.rand(T, H, generator=g) * 2 - 1)).half().to(dev)
    wts = torch.softmax(torch.rand(T, TOPK, generator=g), dim=1).to(dev)
    steps = {}
    for name, fuse in (("unfused", False), ("fused", True)):
        steps[name] = Step(moe.MoEFFN(gate_up, down, qcfg, num_routed=E, fuse_silu=fuse), hidden, ids, wts)
    for s in steps.values():
        s()
    torch.cuda.synchronize()
    same = torch.equal(steps["unfused"].out.view(torch.int16), steps["fused"].out.view(torch.int16))
    print(json.dumps({"check": "fused output bit-identical to unfused", "ok": bool(same)}), flush=True)
    res = {n: {"step": []} | {k: [] for k in s.stages} for n, s in steps.items()}
    for _ in range(args.rounds):
        for n, s in steps.items():
            res[n]["step"].append(time_launches(s, 5, args.iters)["median_ms"])
            for k, fn in s.stages.items():
                res[n][k].append(time_launches(fn, 3, args.iters)["median_ms"])
    for n, d in res.items():
        print(json.dumps({"layer": n, **{k: round(sorted(v)[len(v) // 2] * 1e3, 1) for k, v in d.items()},
                          "unit": "us (median of rounds)", "rounds": d["step"]}), flush=True)
    if not same:
        sys.exit(1)


if __name__ == "__main__":
    main()
