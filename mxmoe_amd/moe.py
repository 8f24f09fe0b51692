"""MoE-layer plumbing around the GroupGEMM, on the C-ABI of include/mxmoe_moe.h.

Reference interface mirrored (SeaCatComplexes/MxMoE, mxmoe/kernels/src/ref_bind.cu, pybind module
``mxmoe_ops``):
  * ``gg_permute_inp(hidden, topk_ids, E)`` ............................ ref_bind.cu:47-64
  * ``quant_inp_act(hidden, topk_ids, num_experts, N, num_shared_experts, qparams_per_exp)``
    -> (inp_list, inp_scale_list, out_list, inp_store, inp_scale_store, out_store,
        recv_tokens_per_exp, perm_indices, dst_exp_sorted) .................. :434-592
  * ``silu_mul_then_quant(inp, num_problems, num_experts, K, N, num_shared_experts, num_tokens, topk,
    values_sorted, recv_tokens_per_exp, qparams_per_exp)``
    -> (inp_list, inp_scale_list, out_list, inp_store, inp_scale_store, out_store) ... :595-757
  * the per-expert quant tag ``cvt_qparams_to_tag`` ...................... :467-479
  * ``gg_unpermute_out`` (an empty stub in the reference, :66) -> ``combine``
and ``MoEFFN``: route -> quant_inp_act -> fused gate_up GroupGEMM -> silu_mul_then_quant -> fused
down GroupGEMM -> combine, the layer the reference's ``gg_mxmoe_share_fused`` path builds toward.

Differences by design: the routing is a device counting sort (mxmoe_moe_route) instead of
torch::sort + bincount; the only host synchronisation is reading the per-expert token counts (the
reference also moves them to the host: ``.cpu()`` at :456), which the tile planner needs anyway.
The quantised activations are written in exactly the GroupGEMM operand layout: pack_wxax rows,
per-token scales [rows] or, for w4a4 g128, [K/128][rows] (permute_scale layout).
"""
from __future__ import annotations

import ctypes
import dataclasses
from typing import Optional, Sequence

import torch

from . import _native as nat
from .groupgemm import GroupGemm, Problem, QParams

ACT_FP16, ACT_INT8, ACT_INT4, ACT_INT4_G128 = 0, 1, 2, 3
_BITS = {ACT_FP16: 16, ACT_INT8: 8, ACT_INT4: 4, ACT_INT4_G128: 4}


def qtag_of(a_bits: int, gsize: int) -> int:
    """The reference's cvt_qparams_to_tag (ref_bind.cu:467-479); unsupported -> ValueError."""
    if a_bits >= 16:
        return ACT_FP16
    if a_bits == 8 and gsize == -1:
        return ACT_INT8
    if a_bits == 4 and gsize == -1:
        return ACT_INT4
    if a_bits == 4 and gsize == 128:
        return ACT_INT4_G128
    raise ValueError(f"activation quantisation a{a_bits} g{gsize} not supported")


def _stream(stream: Optional[torch.cuda.Stream]) -> ctypes.c_void_p:
    s = stream if stream is not None else torch.cuda.current_stream()
    return ctypes.c_void_p(int(s.cuda_stream))


def _ptr(t: Optional[torch.Tensor]) -> Optional[ctypes.c_void_p]:
    return None if t is None else ctypes.c_void_p(t.data_ptr())


@dataclasses.dataclass
class Routing:
    """Result of mxmoe_moe_route: slots sorted by expert (stable in token-major order)."""

    sorted_expert: torch.Tensor  # int32 [T*topk] (the reference's values_sorted / dst_exp_sorted)
    perm_token: torch.Tensor     # int32 [T*topk] (perm_indices)
    inv_slot: torch.Tensor       # int32 [T*topk]: slot of (token t, choice k) at t*topk + k
    counts: list[int]            # host copy of recv_tokens_per_exp [E]
    T: int
    topk: int
    E: int

    @property
    def first_slot(self) -> list[int]:
        out, acc = [], 0
        for c in self.counts:
            out.append(acc)
            acc += c
        return out


def route_device(topk_ids: torch.Tensor, E: int, stream: Optional[torch.cuda.Stream] = None, out=None):
    """The routing launch alone (no host synchronisation): (sorted_expert, perm_token, inv_slot, counts)
    device int32 tensors; `out` reuses a previous result's buffers."""
    if topk_ids.dim() != 2 or topk_ids.dtype != torch.int32 or not topk_ids.is_contiguous():
        raise ValueError("topk_ids must be a contiguous int32 [T, topk] tensor")
    T, topk = topk_ids.shape
    dev = topk_ids.device
    n = T * topk
    if out is None:
        out = tuple(torch.empty(n, dtype=torch.int32, device=dev) for _ in range(3)) + (
            torch.empty(E, dtype=torch.int32, device=dev),)
    nat.check(nat.lib().mxmoe_moe_route(_ptr(topk_ids), T, topk, E, *(_ptr(t) for t in out), _stream(stream)))
    return out


def route(topk_ids: torch.Tensor, E: int, stream: Optional[torch.cuda.Stream] = None) -> Routing:
    """Stable counting sort of the routing choices by expert (one HIP launch + the counts to host)."""
    if topk_ids.dim() != 2:
        raise ValueError("topk_ids must be [T, topk]")
    T, topk = topk_ids.shape
    n = T * topk
    sorted_e, perm, inv, counts = route_device(topk_ids.to(torch.int32).contiguous(), E, stream)
    c = counts.cpu().tolist()
    if sum(c) != n:
        raise ValueError(f"topk_ids holds {n - sum(c)} ids outside [0, {E})")
    return Routing(sorted_e, perm, inv, c, T, topk, E)


@dataclasses.dataclass
class ActBatch:
    """Permuted (and quantised) activations: one segment per expert (+ the shared expert)."""

    out: torch.Tensor     # uint8 store of every segment's rows
    scales: torch.Tensor  # fp16 store of every segment's scales
    segs: list            # nat.MoeSegC per segment (host)
    qtags: list[int]

    def A(self, e: int) -> torch.Tensor:
        """Segment e as the GroupGEMM A operand: fp16 [rows, width] or packed uint8 [rows, width*bits/8]."""
        s = self.segs[e]
        bits = _BITS[self.qtags[e]]
        nbytes = s.rows * s.width * bits // 8
        v = self.out[s.out_off:s.out_off + nbytes]
        if bits == 16:
            return v.view(torch.float16).view(max(s.rows, 0), s.width)
        return v.view(s.rows, s.width * bits // 8)

    def scale(self, e: int) -> Optional[torch.Tensor]:
        s = self.segs[e]
        tag = self.qtags[e]
        if tag == ACT_FP16:
            return None
        n = s.rows * (s.width // 128 if tag == ACT_INT4_G128 else 1)
        return self.scales[s.scale_off:s.scale_off + n]


def _make_segments(rows: Sequence[int], first: Sequence[int], widths: Sequence[int], qtags: Sequence[int],
                   device) -> tuple[list, torch.Tensor, torch.Tensor, torch.Tensor]:
    segs, off, soff = [], 0, 0
    for r, f, w, tag in zip(rows, first, widths, qtags):
        if w % 128:
            raise ValueError(f"segment width {w} must be a multiple of 128")
        segs.append(nat.MoeSegC(tag, f, r, w, off, soff))
        off += (r * w * _BITS[tag] // 8 + 15) // 16 * 16  # 16-B aligned A operands
        soff += 0 if tag == ACT_FP16 else r * (w // 128 if tag == ACT_INT4_G128 else 1)
    arr = (nat.MoeSegC * len(segs))(*segs)
    dev_segs = torch.frombuffer(bytearray(bytes(arr)), dtype=torch.uint8).to(device)
    out = torch.empty(max(off, 16), dtype=torch.uint8, device=device)
    scales = torch.empty(max(soff, 1), dtype=torch.float16, device=device)
    return segs, dev_segs, out, scales


def quant_act(hidden: torch.Tensor, r: Routing, qtags: Sequence[int], with_shared: bool,
              stream: Optional[torch.cuda.Stream] = None) -> ActBatch:
    """Gather hidden rows into expert order and quantise each expert's rows by its tag
    (len(qtags) == E, or E + 1 with the shared expert last)."""
    T, K = hidden.shape
    nseg = r.E + (1 if with_shared else 0)
    if len(qtags) != nseg:
        raise ValueError(f"need {nseg} quant tags, got {len(qtags)}")
    rows = list(r.counts) + ([T] if with_shared else [])
    first = r.first_slot + ([T * r.topk] if with_shared else [])
    segs, dsegs, out, scales = _make_segments(rows, first, [K] * nseg, qtags, hidden.device)
    h = hidden.contiguous()

    def launch(st=stream):
        nat.check(nat.lib().mxmoe_moe_quant_act(_ptr(h), T, K, r.topk, int(with_shared), _ptr(r.sorted_expert),
                                                _ptr(r.perm_token), _ptr(dsegs), nseg, _ptr(out), _ptr(scales),
                                                _stream(st)))

    launch()
    b = ActBatch(out, scales, segs, list(qtags))
    b.relaunch = launch  # same buffers, kernel only (timing / graph capture); keeps h and dsegs alive
    return b


def silu_mul_quant(routed: torch.Tensor, shared: Optional[torch.Tensor], r: Routing, qtags: Sequence[int],
                   stream: Optional[torch.cuda.Stream] = None, activated: bool = False,
                   interleaved: bool = False) -> ActBatch:
    """act = silu(gate) * up of the gate_up outputs (routed [T*topk, 2N] in slot order, shared
    [T, 2Ns]), quantised per expert for the down GroupGEMM. ``activated``: the inputs already are
    the activations (routed [T*topk, N], shared [T, Ns]: the gate_up GroupGEMM's fused SiLU
    epilogue) and only the quantisation runs (mxmoe_moe_quant_slots). ``interleaved``: the gate_up
    output's gate / up columns alternate in 16-column blocks (the fused layout's weights through the
    plain epilogue; mxmoe_moe_silu_mul_quant_il)."""
    div = 1 if activated else 2
    N = routed.shape[1] // div
    Ns = shared.shape[1] // div if shared is not None else 0
    nseg = r.E + (1 if shared is not None else 0)
    if len(qtags) != nseg:
        raise ValueError(f"need {nseg} quant tags, got {len(qtags)}")
    rows = list(r.counts) + ([r.T] if shared is not None else [])
    first = r.first_slot + ([r.T * r.topk] if shared is not None else [])
    widths = [N] * r.E + ([Ns] if shared is not None else [])
    segs, dsegs, out, scales = _make_segments(rows, first, widths, qtags, routed.device)
    fn = (nat.lib().mxmoe_moe_quant_slots if activated else
          nat.lib().mxmoe_moe_silu_mul_quant_il if interleaved else nat.lib().mxmoe_moe_silu_mul_quant)

    def launch(st=stream):
        nat.check(fn(_ptr(routed), _ptr(shared), r.T, r.topk, N, Ns, _ptr(r.sorted_expert), _ptr(dsegs), nseg,
                     _ptr(out), _ptr(scales), _stream(st)))

    launch()
    b = ActBatch(out, scales, segs, list(qtags))
    b.relaunch = launch
    return b


def combine(y: torch.Tensor, r: Routing, weights: torch.Tensor, shared: Optional[torch.Tensor] = None,
            shared_w: Optional[torch.Tensor] = None, stream: Optional[torch.cuda.Stream] = None) -> torch.Tensor:
    """out[t] = sum_k weights[t,k] * y[slot(t,k)] (+ shared_w[t] * shared[t]), f32 fma chain, fp16 out."""
    H = y.shape[1]
    w = weights.to(torch.float32).contiguous()
    sw = None if shared_w is None else shared_w.to(torch.float32).contiguous()
    out = torch.empty(r.T, H, dtype=torch.float16, device=y.device)
    nat.check(nat.lib().mxmoe_moe_combine(_ptr(y), _ptr(r.inv_slot), _ptr(w), _ptr(shared), _ptr(sw), r.T, r.topk, H,
                                          _ptr(out), _stream(stream)))
    return out


def combine_into(out: torch.Tensor, y: torch.Tensor, inv_slot: torch.Tensor, weights: torch.Tensor,
                 shared: Optional[torch.Tensor], topk: int, stream: Optional[torch.cuda.Stream] = None) -> None:
    """combine() on preallocated device buffers (no allocation, one launch: graph-capturable):
    out [T, H] fp16, y [R, H] fp16 rows, inv_slot int32 [T*topk] rows of y, weights f32 [T, topk],
    shared fp16 [T, H] or None. dist.CombineExchange's token-owner combine."""
    T, H = out.shape
    if T == 0:
        return
    nat.check(nat.lib().mxmoe_moe_combine(_ptr(y), _ptr(inv_slot), _ptr(weights), _ptr(shared), None, T, topk, H,
                                          _ptr(out), _stream(stream)))


# ------------------------------------------------------------------ reference-named entry points

def _qtags(qparams_per_exp, n: int) -> list[int]:
    return [qtag_of(int(q[0]), int(q[2])) for q in list(qparams_per_exp)[:n]]


def gg_permute_inp(hidden: torch.Tensor, topk_ids: torch.Tensor, E: int):
    """(num_problems, inp_buffer [T*topk, K] fp16 in expert order, indices, recv_tokens_per_exp)."""
    r = route(topk_ids, E)
    b = quant_act(hidden, r, [ACT_FP16] * E, with_shared=False)
    T, K = hidden.shape
    inp = b.out[: T * r.topk * K * 2].view(torch.float16).view(T * r.topk, K)
    counts = torch.tensor(r.counts, dtype=torch.int64)
    return sum(1 for c in r.counts if c), inp, r.perm_token.to(torch.int64), counts


def quant_inp_act(hidden: torch.Tensor, topk_ids: torch.Tensor, num_experts: int, N: int, num_shared_experts: int,
                  qparams_per_exp, verbose: bool = False):
    """Mirror of ref_bind.cu:434-592. qparams_per_exp[e] = (a_bits, w_bits, gsize, sym), the shared
    expert last. out_store / out_list: the gate_up output buffers (routed [T*topk, 2N] then
    shared [T, 2N * num_shared_experts])."""
    T = hidden.shape[0]
    has_shared = num_shared_experts > 0
    r = route(topk_ids, num_experts)
    tags = _qtags(qparams_per_exp, num_experts + (1 if has_shared else 0))
    b = quant_act(hidden, r, tags, has_shared)
    out_store = torch.empty((num_shared_experts + r.topk) * T * N * 2, dtype=torch.float16, device=hidden.device)
    inp_list, scale_list, out_list = [], [], []
    off = 0
    for e, s in enumerate(b.segs):
        ld = 2 * N * (num_shared_experts if e == num_experts else 1)
        if s.rows == 0:
            continue
        inp_list.append(b.A(e))
        sc = b.scale(e)
        scale_list.append(sc if sc is not None else torch.empty(0, dtype=torch.float16, device=hidden.device))
        out_list.append(out_store[off:off + s.rows * ld].view(s.rows, ld))
        off += s.rows * ld
    if verbose:
        print([(e, s.rows, s.qtag) for e, s in enumerate(b.segs)])
    counts = torch.tensor(r.counts, dtype=torch.int64)
    res = (inp_list, scale_list, out_list, b.out, b.scales, out_store, counts, r.perm_token.to(torch.int64),
           r.sorted_expert)
    return res


def silu_mul_then_quant(inp: torch.Tensor, num_problems: int, num_experts: int, K: int, N: int,
                        num_shared_experts: int, num_tokens: int, topk: int, values_sorted: torch.Tensor,
                        recv_tokens_per_exp: torch.Tensor, qparams_per_exp):
    """Mirror of ref_bind.cu:595-757: inp = the gate_up out_store (routed [T*topk, 2N] then shared
    [T, 2N*S]); returns the quantised down-proj inputs and the down output store [(1+topk)*T*K]."""
    T = num_tokens
    S = num_shared_experts
    routed = inp[: T * topk * 2 * N].view(T * topk, 2 * N)
    shared = inp[T * topk * 2 * N: T * topk * 2 * N + T * 2 * N * S].view(T, 2 * N * S) if S > 0 else None
    counts = [int(c) for c in recv_tokens_per_exp.tolist()]
    r = Routing(values_sorted.to(torch.int32), torch.empty(0), torch.empty(0), counts, T, topk, num_experts)
    tags = _qtags(qparams_per_exp, num_experts + (1 if S > 0 else 0))
    b = silu_mul_quant(routed, shared, r, tags)
    out_store = torch.empty((1 + topk) * T * K, dtype=torch.float16, device=inp.device)
    inp_list, scale_list, out_list = [], [], []
    off = 0
    for e, s in enumerate(b.segs):
        if s.rows == 0:
            continue
        inp_list.append(b.A(e))
        sc = b.scale(e)
        scale_list.append(sc if sc is not None else torch.empty(0, dtype=torch.float16, device=inp.device))
        out_list.append(out_store[off:off + s.rows * K].view(s.rows, K))
        off += s.rows * K
    return inp_list, scale_list, out_list, b.out, b.scales, out_store


_SHARE_FUSED_PLANS: dict = {}


def gg_mxmoe_share_fused(inp: Sequence[torch.Tensor], experts: Sequence[torch.Tensor],
                         scale_zp_a: Sequence[torch.Tensor], scale_zp_b: Sequence[torch.Tensor],
                         output: Sequence[torch.Tensor], N: int, K: int, shared_N: int, shared_K: int,
                         qparams_per_exp, recv_tokens_per_exp: torch.Tensor, verbose: bool = False,
                         stream: Optional[torch.cuda.Stream] = None):
    """Mirror of the reference's fused GroupGEMM op (ref_bind.cu:312-431, pybind name
    ``gg_mxmoe_share_fused``), with its argument meaning:

    * ``recv_tokens_per_exp`` int64 [E] (host or device): routed rows per expert; experts with 0
      rows have no problem. ``experts`` has E entries, or E + 1 with the shared expert last, whose
      problem has ``inp[-1].size(0)`` rows and shape (shared_N, shared_K); routed ones (N, K).
    * ``inp`` / ``scale_zp_a`` / ``output`` are per PROBLEM (non-empty experts in expert order, then
      the shared one), ``experts`` / ``scale_zp_b`` / ``qparams_per_exp`` per EXPERT;
      qparams_per_exp[e] = (a_bits, w_bits, gsize, sym).
    * Operands are in the GroupGEMM layout (the outputs of ``quant_inp_act`` /
      ``silu_mul_then_quant`` and ``prepare_weight``); an empty scale tensor means "no scale" (fp16).

    The reference hard-codes one fused w4a16 + w8a8 kernel (``mxmoe_w4a16_w8a8_bs256``, :412); here
    any supported mix runs on the AUTO variant. The plan (tile table) is cached per shape / qparams
    signature, so repeated calls with the same routing only re-point the operands. Returns ``output``.
    """
    counts = [int(c) for c in recv_tokens_per_exp.tolist()]
    E = len(counts)
    has_shared = len(experts) > E
    num_tokens = int(inp[-1].shape[0]) if len(inp) else 0
    probs = []
    pi = 0
    for e in range(E + (1 if has_shared else 0)):
        rows = num_tokens if e == E else counts[e]
        if rows == 0:
            continue
        if pi >= len(inp):
            raise ValueError(f"gg_mxmoe_share_fused: {len(inp)} inputs for more non-empty experts")
        a_bits, w_bits, gsize, sym = (int(x) for x in qparams_per_exp[e])
        q = QParams(a_bits, w_bits, gsize, bool(sym))
        n, k = (shared_N, shared_K) if e == E else (N, K)

        def opt(t):
            return None if t is None or t.numel() == 0 else t

        C = output[pi]
        probs.append(Problem(A=inp[pi], B=experts[e], C=C, M=rows, N=n, K=k, q=q, scale_a=opt(scale_zp_a[pi]),
                             scale_b=opt(scale_zp_b[e]), ldc=int(C.stride(0)) if C.dim() == 2 else 0))
        if verbose:
            print(f"problem {pi}: [{rows},{n},{k}] qparams: [{a_bits} {w_bits}] {gsize} {int(bool(sym))}")
        pi += 1
    if pi != len(inp):
        raise ValueError(f"gg_mxmoe_share_fused: {len(inp)} inputs for {pi} non-empty experts")
    if not probs:
        return output
    s = stream if stream is not None else torch.cuda.current_stream(probs[0].C.device)
    # one plan per (device, stream, shapes, qparams, strides): a plan's workspace is only ever rebound
    # and launched on its own stream, so a rebind (blocking on that stream) never re-points the
    # operands of a launch still running on another one
    key = (probs[0].C.device, int(s.cuda_stream), tuple((p.M, p.N, p.K, p.q, p.lda, p.ldb, p.ldc) for p in probs))
    gg = _SHARE_FUSED_PLANS.get(key)
    if gg is not None:
        try:
            gg.rebind(probs, stream=s)
        except nat.GGError:  # the library's plan signature disagrees (e.g. a stride the key missed): re-plan
            _evict_share_fused(key)
            gg = None
    if gg is None:
        if len(_SHARE_FUSED_PLANS) >= 64:
            for k in list(_SHARE_FUSED_PLANS):
                _evict_share_fused(k)
        gg = GroupGemm(probs, stream=s)
        gg.stream = s
        if s != torch.cuda.current_stream(gg.device):  # allocated on the current stream, used on s
            gg.workspace.record_stream(s)
        _SHARE_FUSED_PLANS[key] = gg
    gg.launch(s)
    return output


def _evict_share_fused(key) -> None:
    """Drop a cached plan whose launches may still be running on its stream: record the workspace on
    that stream first, so the caching allocator does not hand the memory out before they finish."""
    gg = _SHARE_FUSED_PLANS.pop(key)
    gg.workspace.record_stream(gg.stream)


# ------------------------------------------------------------------ the MoE FFN layer

@dataclasses.dataclass
class ExpertWeights:
    """One linear's GroupGEMM B operand: fp16 [N, K] or packed codes + scale_b, and its QParams."""

    B: torch.Tensor
    scale_b: Optional[torch.Tensor]
    q: QParams
    N: int
    K: int


def prepare_weight(w: torch.Tensor, q: QParams, interleave: bool = False) -> ExpertWeights:
    """fp16 [N, K] -> the GroupGEMM's B operand for qcfg q (setup, once per weight). interleave: a
    gate_up weight ([gate; up] rows) reordered for the fused SiLU epilogue (interleave_gate_up; the
    per-row scales follow their rows)."""
    from .groupgemm import interleave_gate_up
    from .quantize import pack_weightonly_mi355x, pack_wxax, quant_rtn_sym, quant_weightonly

    N, K = w.shape
    if interleave:
        w = interleave_gate_up(w)[0]  # (per-row quantisation commutes with the row order)
    if not q.is_quant:
        return ExpertWeights(w.contiguous(), None, q, N, K)
    if q.is_weight_only:
        codes, sz = quant_weightonly(w, q.w_bits, q.gsize, q.sym)
        return ExpertWeights(pack_weightonly_mi355x(codes, q.w_bits), sz, q, N, K)
    qw, sw = quant_rtn_sym(w, q.w_bits, q.gsize)
    return ExpertWeights(pack_wxax(qw, q.w_bits), sw, q, N, K)


class MoEFFN:
    """A quantised MoE FFN layer (routed experts + optional shared expert) on the fused GroupGEMM.

    gate_up[e]: fp16 [2N, H] (gate rows then up rows), down[e]: fp16 [H, N]; qcfg[e] = (QParams of
    gate_up, QParams of down) — the activation side (a_bits, gsize) of each QParams sets how the
    plumbing quantises that expert's input (qtag_of). Expert E (if given) is the shared expert."""

    # gate_up qcfgs with the SiLU epilogue: fp16 / w8a8 / w4a4 on every product kernel, weight-only
    # on the small-batch kernel (wo3; a large call of those falls back to the interleaved form)
    FUSE_QCFGS = ("fp16", "w8a8_g-1_sym", "w4a4_g-1_sym")
    FUSE_WEIGHT_ONLY = True

    def __init__(self, gate_up: Sequence[torch.Tensor], down: Sequence[torch.Tensor],
                 qcfg: Sequence[tuple[QParams, QParams]], num_routed: int, fuse_silu: Optional[bool] = None):
        """fuse_silu: the gate_up GroupGEMM writes act = silu(gate) * up straight from its epilogue
        (MXMOE_GG_EPI_SILU_MUL; gate_up weights stored with gate / up rows interleaved in 16-row
        blocks) and only the quantisation runs after it — bit-identical outputs, half the gate_up C
        bytes and no separate SiLU pass (qwen2_moe layer step -6 %). Needs every gate_up qcfg in
        FUSE_QCFGS. None (default): fuse whenever the qcfgs allow. A call whose kernel has no SiLU
        epilogue (lab kernels; ``gate_up_mode = "interleaved"`` forces it) runs the plain epilogue on
        the interleaved weights and the interleaved-input SiLU pass instead — same outputs. (Before
        round 6 that was every small-batch call: the wo3 kernel's fp16 / w8a8 / w4a4 bodies now carry
        the epilogue too.)"""
        self.E = num_routed
        self.has_shared = len(gate_up) == num_routed + 1
        self.H = gate_up[0].shape[1]
        self.N = gate_up[0].shape[0] // 2
        self.Ns = gate_up[-1].shape[0] // 2 if self.has_shared else 0
        self.qcfg = list(qcfg)
        eligible = all(q[0].qcfg in self.FUSE_QCFGS or (self.FUSE_WEIGHT_ONLY and q[0].is_weight_only) for q in qcfg)
        if fuse_silu and not eligible:
            raise ValueError(f"fuse_silu needs every gate_up qcfg in {self.FUSE_QCFGS} or weight-only")
        self.fuse_silu = eligible if fuse_silu is None else fuse_silu
        self.w1 = [prepare_weight(w, q[0], interleave=self.fuse_silu) for w, q in zip(gate_up, qcfg)]
        self.w2 = [prepare_weight(w, q[1]) for w, q in zip(down, qcfg)]
        self.tag1 = [qtag_of(q[0].a_bits, q[0].gsize) for q in qcfg]
        self.tag2 = [qtag_of(q[1].a_bits, q[1].gsize) for q in qcfg]
        self.gate_up_mode: Optional[str] = None  # None: the library decides; "interleaved": A/B override

    def gate_up_call(self, a1: ActBatch, T: int, topk: int, dev):
        """The planned gate_up GroupGEMM of one call and its output buffers: (GroupGemm, h1, h1s, mode),
        mode "plain" ([gate | up] columns), "fused" (the SiLU epilogue: N-wide activations) or
        "interleaved" (fused-layout weights through the plain epilogue and the interleaved-input SiLU
        pass, for calls whose kernel has no SiLU epilogue). The library decides: the variant AUTO
        resolves the call's shapes to is asked for MXMOE_GG_CAP_SILU_MUL (mxmoe_gg_variant_caps), and
        a fused plan the library still refuses (GGError UNSUPPORTED) falls back to "interleaved"."""
        def problems(C_of, silu):
            ps = []
            for e, sg in enumerate(a1.segs):
                if sg.rows:
                    w = self.w1[e]
                    ps.append(Problem(A=a1.A(e), B=w.B, C=C_of(e, sg), M=sg.rows, N=w.N, K=w.K, q=w.q,
                                      scale_a=a1.scale(e), scale_b=w.scale_b, silu=silu))
            return ps

        def buffers(mode):
            f = 1 if mode == "fused" else 2
            h1 = torch.empty(T * topk, f * self.N, dtype=torch.float16, device=dev)
            h1s = torch.empty(T, f * self.Ns, dtype=torch.float16, device=dev) if self.has_shared else None
            ps = problems(lambda e, sg: h1s if e == self.E else h1[sg.first_slot:sg.first_slot + sg.rows],
                          mode == "fused")
            return ps, h1, h1s

        if self.gate_up_mode not in (None, "interleaved"):
            raise ValueError(f"gate_up_mode must be None or 'interleaved', got {self.gate_up_mode!r}")
        mode = "plain"
        if self.fuse_silu and self.gate_up_mode == "interleaved":
            mode = "interleaved"
        elif self.fuse_silu:
            ph = torch.empty(0, dtype=torch.float16, device=dev)
            probe = problems(lambda e, sg: ph, False)  # shapes only: AUTO's choice for the plain epilogue
            arr = (nat.GGProblemC * max(len(probe), 1))(*[p.to_c() for p in probe])
            v = nat.resolve_variant(arr, len(probe))
            mode = "fused" if nat.variant_caps(v) & nat.CAP_SILU_MUL else "interleaved"
        if mode == "fused":
            ps, h1, h1s = buffers(mode)
            try:
                return GroupGemm(ps, device=dev), h1, h1s, mode
            except nat.GGError as e:
                if e.status != nat.MXMOE_GG_ERR_UNSUPPORTED:
                    raise
                mode = "interleaved"
        ps, h1, h1s = buffers(mode)
        return GroupGemm(ps, device=dev), h1, h1s, mode

    def forward(self, hidden: torch.Tensor, topk_ids: torch.Tensor, topk_weights: torch.Tensor,
                shared_w: Optional[torch.Tensor] = None, return_intermediates: bool = False):
        T = hidden.shape[0]
        dev = hidden.device
        r = route(topk_ids, self.E)
        topk = r.topk
        a1 = quant_act(hidden, r, self.tag1, self.has_shared)
        g1, h1, h1s, mode = self.gate_up_call(a1, T, topk, dev)
        g1.launch()
        a2 = silu_mul_quant(h1, h1s, r, self.tag2, activated=mode == "fused", interleaved=mode == "interleaved")
        y = torch.empty(T * topk, self.H, dtype=torch.float16, device=dev)
        ys = torch.empty(T, self.H, dtype=torch.float16, device=dev) if self.has_shared else None
        probs = []
        for e, s in enumerate(a2.segs):
            if s.rows == 0:
                continue
            w = self.w2[e]
            C = ys if e == self.E else y[s.first_slot:s.first_slot + s.rows]
            probs.append(Problem(A=a2.A(e), B=w.B, C=C, M=s.rows, N=w.N, K=w.K, q=w.q, scale_a=a2.scale(e),
                                 scale_b=w.scale_b))
        GroupGemm(probs, device=dev).launch()
        out = combine(y, r, topk_weights, ys, shared_w)
        if return_intermediates:
            return out, dict(routing=r, a1=a1, h1=h1, h1s=h1s, a2=a2, y=y, ys=ys)
        return out




class PlannedForward:
    """MoEFFN.forward for a fixed routing with every launch planned once: the plumbing kernels
    relaunch on the same buffers and both GroupGEMMs keep their plans (the device work of a serving
    step whose routing shapes repeat; the host planning MoEFFN.forward redoes per call is left out).
    ``stages`` maps stage name -> launch; calling the object runs them in order into ``out``."""

    def __init__(self, layer: "MoEFFN", hidden: torch.Tensor, topk_ids: torch.Tensor, topk_weights: torch.Tensor):
        dev = hidden.device
        T = hidden.shape[0]
        self.r = r = route(topk_ids, layer.E)
        topk = r.topk
        self.a1 = quant_act(hidden, r, layer.tag1, layer.has_shared)
        self.g1, self.h1, self.h1s, self.mode = layer.gate_up_call(self.a1, T, topk, dev)
        self.a2 = silu_mul_quant(self.h1, self.h1s, r, layer.tag2, activated=self.mode == "fused",
                                 interleaved=self.mode == "interleaved")
        self.y = torch.empty(T * topk, layer.H, dtype=torch.float16, device=dev)
        self.ys = torch.empty(T, layer.H, dtype=torch.float16, device=dev) if layer.has_shared else None
        p2 = []
        for e, sg in enumerate(self.a2.segs):
            if sg.rows:
                w = layer.w2[e]
                C = self.ys if e == layer.E else self.y[sg.first_slot:sg.first_slot + sg.rows]
                p2.append(Problem(A=self.a2.A(e), B=w.B, C=C, M=sg.rows, N=w.N, K=w.K, q=w.q, scale_a=self.a2.scale(e),
                                  scale_b=w.scale_b))
        self.g2 = GroupGemm(p2, device=dev)
        self.out = torch.empty(T, layer.H, dtype=torch.float16, device=dev)
        self.w = topk_weights.to(torch.float32).contiguous()
        self.stages = {"quant_act": self.a1.relaunch, "gate_up": self.g1.launch, "act_quant": self.a2.relaunch,
                       "down": self.g2.launch,
                       "combine": lambda: combine_into(self.out, self.y, r.inv_slot, self.w, self.ys, topk)}

    def __call__(self) -> torch.Tensor:
        for fn in self.stages.values():
            fn()
        return self.out


def qwen2_layer_bench(rounds: int = 4, iters: int = 30, bs: int = 8192, model: str = "qwen2_moe",
                      interleaved: bool = False, scheme: str = "lp1") -> dict:
    """qwen2_moe layer 11 (LP-1 mixed w4a4 + w8a8 qconfig, the committed routing histogram) — or
    model="ds2": the DeepSeek-V2-Lite mixed layer of the bench (64 routed experts, top-6, the two
    shared experts as one of twice the width) — with random weights, as planned MoE FFN steps,
    unfused vs the fused SiLU epilogue: per-stage and step device times (median over alternating
    rounds, µs) and whether the two outputs are bit-identical. interleaved: a third step, the fused
    layout through the plain epilogue + the interleaved-input SiLU pass (the small-batch form before
    round 6), with each step's gate_up mode. scheme (qwen2_moe): "lp1" (the LP-1 mixed w4a4 + w8a8
    qconfig) or "w4a16_w8a8" (the reference's small-batch scheme, hz_fused.cuh:14-125)."""
    from .harness import time_launches
    from .workload import (ds2_mixed_qconfig, ds2_workload, load_workload, mixed_qconfig_lp1, qwen2_layer11_workload,
                           w4a16_w8a8_qconfig)

    if model == "ds2":
        layer = load_workload(ds2_workload(bs, qconfig=ds2_mixed_qconfig()))["layer-1"]
    else:
        qc = w4a16_w8a8_qconfig() if scheme == "w4a16_w8a8" else mixed_qconfig_lp1()
        layer = load_workload(qwen2_layer11_workload(bs, qconfig=qc))["layer-11"]
    E = len(layer["gate_up"]) - 1
    H = layer["gate_up"][0].K
    N, Ns = layer["down"][0].K, layer["down"][-1].K
    topk = max(1, round(sum(s.M for s in layer["gate_up"][:E]) / bs))
    qcfg = [(QParams(a.a_bits, a.w_bits, a.gsize, a.sym), QParams(b.a_bits, b.w_bits, b.gsize, b.sym))
            for a, b in zip(layer["gate_up"], layer["down"])]
    counts = [s.M for s in layer["gate_up"][:E]]
    counts[0] += bs * topk - sum(counts)  # the histogram's int() truncation
    dev = "cuda"
    g = torch.Generator().manual_seed(0)
    ids = torch.repeat_interleave(torch.arange(E, dtype=torch.int32), torch.tensor(counts))
    ids = ids[torch.randperm(ids.numel(), generator=g)].view(bs, topk).contiguous().to(dev)
    gate_up = [((torch.rand(2 * N, H, generator=g) * 2 - 1) * 0.05).half().to(dev) for _ in range(E)]
    gate_up.append(((torch.rand(2 * Ns, H, generator=g) * 2 - 1) * 0.05).half().to(dev))
    down = [((torch.rand(H, N, generator=g) * 2 - 1) * 0.05).half().to(dev) for _ in range(E)]
    down.append(((torch.rand(H, Ns, generator=g) * 2 - 1) * 0.05).half().to(dev))
    hidden = ((torch.rand(bs, H, generator=g) * 2 - 1)).half().to(dev)
    wts = torch.softmax(torch.rand(bs, topk, generator=g), dim=1).to(dev)
    modes = [("unfused", False, None), ("fused", True, None)] + ([("interleaved", True, "interleaved")] if interleaved else [])
    steps = {}
    for name, fuse, override in modes:
        layer_ = MoEFFN(gate_up, down, qcfg, num_routed=E, fuse_silu=fuse)
        layer_.gate_up_mode = override
        steps[name] = PlannedForward(layer_, hidden, ids, wts)
    del gate_up, down, layer_
    for st in steps.values():
        st()
    torch.cuda.synchronize()
    same = all(torch.equal(steps["unfused"].out.view(torch.int16), st.out.view(torch.int16)) for st in steps.values())
    res = {n: {"step": []} | {k: [] for k in st.stages} for n, st in steps.items()}
    for _ in range(rounds):
        for n, st in steps.items():
            res[n]["step"].append(time_launches(st, 5, iters)["median_ms"])
            for k, fn in st.stages.items():
                res[n][k].append(time_launches(fn, 3, iters)["median_ms"])
    out = {n: {k: round(sorted(v)[len(v) // 2] * 1e3, 1) for k, v in d.items()} for n, d in res.items()}
    out["bit_identical"] = bool(same)
    out["speedup"] = round(out["unfused"]["step"] / out["fused"]["step"], 4)
    out["gate_up_mode"] = {n: st.mode for n, st in steps.items()}
    names = [ln.split()[1] for ln in nat.list_variants()]
    out["gate_up_variant"] = {n: names[st.g1.variant] for n, st in steps.items()}
    return out
