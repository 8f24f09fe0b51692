"""The bit identities behind wo3's code -> fp16 step (gg_device.h `WoK` / `wo_dequant`, WO_NIBPOS):
a 4-bit code ORed into the mantissa at bits 0-3 of fp16 1024.0, or at bits 4-7 of fp16 64.0, and a
2-bit code at bits 0 / 2 / 4 / 6 of 1024 / 256 / 64 / 16, reads as base + u exactly; subtracting
base + off is exact, so fma(x, s, z) sees the same x = u - off whichever position the code sat in
(the round-3 form shifted every code down to bits 0-3 first). CPU only: numpy's fp16 is IEEE
binary16, as the hardware's."""
from __future__ import annotations

import numpy as np

BASES4 = {0: (0x6400, 1024.0), 4: (0x5400, 64.0)}
BASES2 = {0: (0x6400, 1024.0), 2: (0x5C00, 256.0), 4: (0x5400, 64.0), 6: (0x4C00, 16.0)}


def _f16(bits: int) -> float:
    return float(np.array([bits], dtype=np.uint16).view(np.float16)[0])


def _check(bases, width):
    for shift, (magic, base) in bases.items():
        assert _f16(magic) == base
        for off in (0, (1 << (width - 1)) - 1):  # asym, sym (7 for 4-bit, 1 for 2-bit)
            sub = np.float16(-(base + off))
            assert float(sub) == -(base + off)  # the subtrahend is exact
            for u in range(1 << width):
                d = np.float16(_f16(magic | (u << shift)))
                assert float(d) == base + u
                x = np.float16(d + sub)  # one fp16 add, as v_pk_add_f16
                assert float(x) == u - off


def test_4bit_positions_read_exactly():
    _check(BASES4, 4)


def test_2bit_positions_read_exactly():
    _check(BASES2, 2)


def test_fma_after_either_position_rounds_identically():
    rng = np.random.default_rng(3)
    s = rng.uniform(1e-4, 0.2, 256).astype(np.float16)
    z = rng.uniform(-1, 1, 256).astype(np.float16)
    for u in range(16):
        x_lo = np.float16(np.float16(_f16(0x6400 | u)) + np.float16(-1024.0))
        x_hi = np.float16(np.float16(_f16(0x5400 | (u << 4))) + np.float16(-64.0))
        assert x_lo == x_hi == u
        # fma with one rounding (float64 holds the exact product + sum of fp16 operands)
        r_lo = (np.float64(x_lo) * s.astype(np.float64) + z.astype(np.float64)).astype(np.float16)
        r_hi = (np.float64(x_hi) * s.astype(np.float64) + z.astype(np.float64)).astype(np.float16)
        assert np.array_equal(r_lo.view(np.uint16), r_hi.view(np.uint16))
