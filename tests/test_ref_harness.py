"""The reference-side C++ boundary, compiled (VERDICT r03 missing #3): tests/cpp/ref_harness_call is a
hipcc-built program that declares the reference's registry FuncType (half**, dim3*, QParams*;
registry.cuh:28-39), registers groupgemm_mxmoe in a registry table as INTEGRATION.md §2 shows, builds
its operand arrays like the reference harness (test.cu:488-554: one buffer per operand, scale_zp =
[sa(M) | sb(N)] per problem, QParams padding left as garbage) and calls through the function pointer
(test.cu:793-813). CPU: the layouts agree (static_asserts in tests/cpp/layout_check.cpp compiled, and
the program's own report). GPU: a mixed fp16 / w8a8 / w4a4 golden call, quantised problems bit-exact.
"""
from __future__ import annotations

import json
import subprocess
from pathlib import Path

import numpy as np
import pytest

from mxmoe_amd import build as b
from tests._util import assert_f16_close

GOLD = Path(__file__).resolve().parent / "golden"


def _harness() -> Path:
    exe = b.REF_HARNESS
    if not exe.exists():
        pytest.fail(f"{exe} missing: build it with __graft_entry__.build() (mxmoe_amd.build.build_ref_harness)")
    return exe


def test_reference_side_layouts_match():
    r = subprocess.run([str(_harness()), "--layout"], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stderr
    lay = json.loads(r.stdout)
    # mxmoe_qparams (include/mxmoe_gg.h): 16 B, 8-B aligned, gsize at 8, sym at 12; dim3 = 3 x u32
    assert lay == {"sizeof_QParams": 16, "alignof_QParams": 8, "offsetof_gsize": 8, "offsetof_sym": 12,
                   "sizeof_dim3": 12, "sizeof_half": 2, "layout_check": 1, "registered": 1}


def _write_input(path: Path, d) -> list:
    P = int(d["P"])
    heads, blobs, probs = [], [], []
    for i in range(P):
        M, N, K = (int(x) for x in d[f"p{i}_shape"])
        bits = int(d[f"p{i}_bits"])
        q = bits < 16
        heads.append(np.array([M, N, K, bits, bits, -1, 1 if q else 0], dtype=np.int32))
        parts = [np.ascontiguousarray(d[f"p{i}_A"]), np.ascontiguousarray(d[f"p{i}_B"])]
        if q:
            parts += [d[f"p{i}_sa"].astype(np.float16), d[f"p{i}_sb"].astype(np.float16)]
        blobs.append(b"".join(p.tobytes() for p in parts))
        probs.append((M, N, K, q))
    with open(path, "wb") as f:
        f.write(np.int32(P).tobytes())
        for h in heads:
            f.write(h.tobytes())
        for bl in blobs:
            f.write(bl)
    return probs


@pytest.mark.gpu
def test_reference_harness_runs_mixed_call_through_funcptr(tmp_path):
    d = np.load(GOLD / "gg_mixed_small.npz")
    probs = _write_input(tmp_path / "in.bin", d)
    assert {q for *_, q in probs} == {True, False} and {int(d[f"p{i}_bits"]) for i in range(int(d["P"]))} >= {4, 8, 16}
    r = subprocess.run([str(_harness()), str(tmp_path / "in.bin"), str(tmp_path / "out.bin")],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert json.loads(r.stdout.strip().splitlines()[-1]) == {"ran": 1, "problems": int(d["P"])}
    out = np.fromfile(tmp_path / "out.bin", dtype=np.float16)
    off = 0
    for i, (M, N, K, q) in enumerate(probs):
        got = out[off:off + M * N].reshape(M, N)
        off += M * N
        if q:
            ref = d[f"p{i}_C"]
            assert (got.view(np.uint16) == ref.view(np.uint16)).all(), f"problem {i} ({M}x{N}x{K})"
        else:
            assert_f16_close(got, d[f"p{i}_C_f64"], K)
    assert off == out.size
