"""ctypes binding of ``libmxmoe_gg.so`` (the C-ABI in ``include/mxmoe_gg.h``).

The library is the product path: if it is missing or does not load, every GPU entry point raises
``NativeLibraryError`` — there is no CPU or PyTorch fallback anywhere in the package.

torch is imported before the library is opened so that ``libamdhip64.so.7`` resolves to the HIP
runtime torch already loaded (one runtime per process; streams and device pointers are shared).
"""
from __future__ import annotations

import atexit
import ctypes
import os
from pathlib import Path

import torch  # noqa: F401  (must precede the CDLL: binds the shared HIP runtime)

LIB_DIR = Path(__file__).resolve().parent / "lib"
LIB_PATH = LIB_DIR / "libmxmoe_gg.so"

MXMOE_GG_OK = 0
MXMOE_GG_ERR_INVALID = 1
MXMOE_GG_ERR_UNSUPPORTED = 2
MXMOE_GG_ERR_WORKSPACE = 3
MXMOE_GG_ERR_HIP = 4

# operand formats (MXMOE_GG_FMT_*): fp16 / integer, OCP fp8 e4m3, bfloat16; FMT_F6 (w4a4 as fp6
# images, gg_f6.h) is understood by the lab library only (measured slower)
FMT_DEFAULT, FMT_E4M3, FMT_BF16, FMT_F6 = 0, 1, 2, 3
EPI_SILU_MUL = 0x100  # MXMOE_GG_EPI_SILU_MUL: fmt flag, C = silu(gate) * up (include/mxmoe_gg.h)


def f6_row_bytes(K: int) -> int:
    """Bytes of one fp6-image row of K int4 codes (96 per K-128 block; lab library)."""
    return (K + 127) // 128 * 96


class NativeLibraryError(RuntimeError):
    """libmxmoe_gg.so is missing or failed to load."""


class GGError(RuntimeError):
    """A C-ABI call returned a non-zero status."""

    def __init__(self, status: int, message: str):
        super().__init__(f"mxmoe_gg status {status}: {message}")
        self.status = status


class MxmoeQParams(ctypes.Structure):
    """Layout of the reference's mxmoe::QParams (quantize.cuh:14-25): int2 qbits; int gsize; bool sym."""

    _fields_ = [("a_bits", ctypes.c_int32), ("w_bits", ctypes.c_int32), ("gsize", ctypes.c_int32),
                ("sym", ctypes.c_uint8), ("pad_", ctypes.c_uint8 * 3)]


class MxmoeDim3(ctypes.Structure):
    _fields_ = [("x", ctypes.c_uint32), ("y", ctypes.c_uint32), ("z", ctypes.c_uint32)]


class GGProblemC(ctypes.Structure):
    _fields_ = [
        ("A", ctypes.c_void_p), ("B", ctypes.c_void_p), ("scale_a", ctypes.c_void_p),
        ("scale_b", ctypes.c_void_p), ("C", ctypes.c_void_p),
        ("M", ctypes.c_int32), ("N", ctypes.c_int32), ("K", ctypes.c_int32),
        ("a_bits", ctypes.c_int32), ("w_bits", ctypes.c_int32), ("gsize", ctypes.c_int32),
        ("sym", ctypes.c_int32), ("fmt", ctypes.c_int32),
        ("lda", ctypes.c_int64), ("ldb", ctypes.c_int64), ("ldc", ctypes.c_int64),
    ]


VARIANT_AUTO = -1  # MXMOE_GG_VARIANT_AUTO
CAP_SILU_MUL = 1  # MXMOE_GG_CAP_SILU_MUL (mxmoe_gg_variant_caps)
ABI_VERSION = 7  # MXMOE_GG_ABI_VERSION this binding is written for (include/mxmoe_gg.h)


class GGPlanInfo(ctypes.Structure):
    _fields_ = [
        ("variant", ctypes.c_int32), ("problem_count", ctypes.c_int32), ("total_tiles", ctypes.c_int32),
        ("grid", ctypes.c_int32), ("block", ctypes.c_int32), ("lds_bytes", ctypes.c_int32),
        ("qtype_mask", ctypes.c_int32), ("splitk_slabs", ctypes.c_int32), ("workspace_bytes", ctypes.c_int64), ("workspace", ctypes.c_void_p),
        ("signature", ctypes.c_uint64), ("tile_slots", ctypes.c_int32), ("reserved", ctypes.c_int32),
    ]


# every symbol include/mxmoe_gg.h declares (tests check the .so exports exactly these)
EXPORTED_SYMBOLS = (
    "mxmoe_gg_abi_version", "mxmoe_gg_last_error", "mxmoe_gg_variant_count", "mxmoe_gg_default_variant",
    "mxmoe_gg_list_variants",
    "mxmoe_gg_variant_tile", "mxmoe_gg_variant_caps", "mxmoe_gg_resolve_variant", "mxmoe_gg_workspace_size", "mxmoe_gg_plan", "mxmoe_gg_rebind", "mxmoe_gg_forget_workspace", "mxmoe_gg_launch", "mxmoe_gg_run",
    "groupgemm_mxmoe", "groupgemm_mxmoe_fmt", "mxmoe_gg_release_shim_workspaces", "mxmoe_gg_repack_weightonly", "mxmoe_gg_debug_trace",
    "mxmoe_gg_plan_tiles",
    # include/mxmoe_moe.h (MoE-layer plumbing)
    "mxmoe_moe_route", "mxmoe_moe_quant_act", "mxmoe_moe_silu_mul_quant", "mxmoe_moe_silu_mul_quant_il", "mxmoe_moe_quant_slots", "mxmoe_moe_combine",
)


class MoeSegC(ctypes.Structure):
    """mxmoe_moe_seg (include/mxmoe_moe.h): one expert's segment of a permuted activation buffer."""

    _fields_ = [("qtag", ctypes.c_int32), ("first_slot", ctypes.c_int32), ("rows", ctypes.c_int32),
                ("width", ctypes.c_int32), ("out_off", ctypes.c_int64), ("scale_off", ctypes.c_int64)]

_lib = None


def _declare(lib: ctypes.CDLL) -> None:
    c = ctypes
    lib.mxmoe_gg_abi_version.restype = c.c_int
    lib.mxmoe_gg_abi_version.argtypes = []
    lib.mxmoe_gg_last_error.restype = c.c_char_p
    lib.mxmoe_gg_last_error.argtypes = []
    lib.mxmoe_gg_variant_count.restype = c.c_int
    lib.mxmoe_gg_variant_count.argtypes = []
    lib.mxmoe_gg_default_variant.restype = c.c_int
    lib.mxmoe_gg_default_variant.argtypes = []
    lib.mxmoe_gg_list_variants.restype = c.c_int
    lib.mxmoe_gg_list_variants.argtypes = [c.c_char_p, c.c_size_t]
    lib.mxmoe_gg_variant_tile.restype = c.c_int
    lib.mxmoe_gg_variant_tile.argtypes = [c.c_int, c.c_int, c.c_int] + [c.POINTER(c.c_int32)] * 4
    lib.mxmoe_gg_resolve_variant.restype = c.c_int
    lib.mxmoe_gg_resolve_variant.argtypes = [c.POINTER(GGProblemC), c.c_int, c.c_int, c.POINTER(c.c_int)]
    lib.mxmoe_gg_workspace_size.restype = c.c_int
    lib.mxmoe_gg_workspace_size.argtypes = [c.POINTER(GGProblemC), c.c_int, c.c_int, c.POINTER(c.c_size_t)]
    lib.mxmoe_gg_plan.restype = c.c_int
    lib.mxmoe_gg_plan.argtypes = [c.POINTER(GGProblemC), c.c_int, c.c_int, c.c_void_p, c.c_size_t, c.c_void_p,
                                  c.POINTER(GGPlanInfo)]
    lib.mxmoe_gg_rebind.restype = c.c_int
    lib.mxmoe_gg_rebind.argtypes = [c.POINTER(GGProblemC), c.c_int, c.POINTER(GGPlanInfo), c.c_void_p]
    if hasattr(lib, "mxmoe_gg_forget_workspace"):  # (ABI 6+; older builds loaded by A/B tools lack it)
        lib.mxmoe_gg_forget_workspace.restype = c.c_int
        lib.mxmoe_gg_forget_workspace.argtypes = [c.c_void_p]
    if hasattr(lib, "mxmoe_gg_variant_caps"):  # (ABI 7+)
        lib.mxmoe_gg_variant_caps.restype = c.c_int
        lib.mxmoe_gg_variant_caps.argtypes = [c.c_int, c.POINTER(c.c_uint32)]
    lib.mxmoe_gg_launch.restype = c.c_int
    lib.mxmoe_gg_launch.argtypes = [c.POINTER(GGPlanInfo), c.c_void_p]
    lib.mxmoe_gg_run.restype = c.c_int
    lib.mxmoe_gg_run.argtypes = [c.POINTER(GGProblemC), c.c_int, c.c_int, c.c_void_p, c.c_size_t, c.c_void_p]
    lib.groupgemm_mxmoe.restype = c.c_int
    lib.groupgemm_mxmoe.argtypes = [c.c_void_p] * 10 + [c.c_void_p, c.POINTER(MxmoeDim3), c.c_void_p,
                                                         c.POINTER(MxmoeQParams), c.c_int]
    lib.groupgemm_mxmoe_fmt.restype = c.c_int
    lib.groupgemm_mxmoe_fmt.argtypes = lib.groupgemm_mxmoe.argtypes + [c.c_void_p]
    lib.mxmoe_gg_release_shim_workspaces.restype = c.c_int
    lib.mxmoe_gg_release_shim_workspaces.argtypes = []
    lib.mxmoe_gg_repack_weightonly.restype = c.c_int
    lib.mxmoe_gg_repack_weightonly.argtypes = [c.c_void_p, c.c_int, c.c_int, c.c_int, c.c_void_p]
    lib.mxmoe_gg_debug_trace.restype = c.c_int
    lib.mxmoe_gg_debug_trace.argtypes = [c.c_void_p, c.c_size_t, c.c_int]
    lib.mxmoe_gg_plan_tiles.restype = c.c_int
    lib.mxmoe_gg_plan_tiles.argtypes = [c.POINTER(GGProblemC), c.c_int, c.c_int, c.c_void_p, c.c_void_p,
                                        c.POINTER(c.c_int)]
    if hasattr(lib, "mxmoe_gg_pack_f6"):  # lab library only
        lib.mxmoe_gg_pack_f6.restype = c.c_int
        lib.mxmoe_gg_pack_f6.argtypes = [c.c_void_p, c.c_int, c.c_int, c.c_int64, c.c_void_p, c.c_int64, c.c_void_p]
        lib.mxmoe_gg_pack_f6_host.restype = c.c_int
        lib.mxmoe_gg_pack_f6_host.argtypes = [c.c_void_p, c.c_int, c.c_int, c.c_int64, c.c_void_p, c.c_int64]
    P = c.c_void_p
    lib.mxmoe_moe_route.restype = c.c_int
    lib.mxmoe_moe_route.argtypes = [P, c.c_int64, c.c_int, c.c_int, P, P, P, P, P]
    lib.mxmoe_moe_quant_act.restype = c.c_int
    lib.mxmoe_moe_quant_act.argtypes = [P, c.c_int64, c.c_int, c.c_int, c.c_int, P, P, P, c.c_int, P, P, P]
    lib.mxmoe_moe_silu_mul_quant.restype = c.c_int
    lib.mxmoe_moe_silu_mul_quant.argtypes = [P, P, c.c_int64, c.c_int, c.c_int, c.c_int, P, P, c.c_int, P, P, P]
    for fn in ("mxmoe_moe_quant_slots", "mxmoe_moe_silu_mul_quant_il"):
        if hasattr(lib, fn):  # (builds before round 5's fused SiLU epilogue lack them: A/B tools)
            getattr(lib, fn).restype = c.c_int
            getattr(lib, fn).argtypes = [P, P, c.c_int64, c.c_int, c.c_int, c.c_int, P, P, c.c_int, P, P, P]
    lib.mxmoe_moe_combine.restype = c.c_int
    lib.mxmoe_moe_combine.argtypes = [P, P, P, P, P, c.c_int64, c.c_int, c.c_int, P, P]


def lib() -> ctypes.CDLL:
    """The loaded library; raises NativeLibraryError (never falls back)."""
    global _lib
    if _lib is None:
        path = Path(os.environ.get("MXMOE_GG_LIB", LIB_PATH))
        if not path.exists():
            raise NativeLibraryError(
                f"{path} not found: build it with `python -c 'import __graft_entry__ as g; g.build()'` "
                "(hipcc --offload-arch=gfx950). There is no fallback path.")
        try:
            handle = ctypes.CDLL(str(path))
        except OSError as e:  # pragma: no cover - environment dependent
            raise NativeLibraryError(f"failed to load {path}: {e}") from e
        _check_abi(handle, path)
        _declare(handle)
        _lib = handle
        atexit.register(_release_shim)
    return _lib


def _check_abi(handle: ctypes.CDLL, path: Path) -> None:
    """The product library must carry the ABI this binding is written for (a stale or foreign .so
    raises NativeLibraryError here, not an AttributeError or a mis-typed call later). A library
    named by MXMOE_GG_LIB (the A/B tools' older or lab builds) may be older: the symbols added
    since are bound only where present."""
    try:
        fn = handle.mxmoe_gg_abi_version
    except AttributeError as e:
        raise NativeLibraryError(f"{path} exports no mxmoe_gg_abi_version: not a libmxmoe_gg build") from e
    fn.restype, fn.argtypes = ctypes.c_int, []
    got = fn()
    if got == ABI_VERSION or ("MXMOE_GG_LIB" in os.environ and 5 <= got < ABI_VERSION):
        return
    raise NativeLibraryError(f"{path} has ABI version {got}, this binding needs {ABI_VERSION}: rebuild it with "
                             "`python -c 'import __graft_entry__ as g; g.build()'`")


def _release_shim() -> None:
    """Free the reference-ABI shim's per-device buffers before the HIP runtime tears down (only if
    a GPU is present: on a CPU-only host no shim call can have allocated)."""
    try:
        import torch

        if torch.cuda.is_initialized():
            _lib.mxmoe_gg_release_shim_workspaces()
    except Exception:  # pragma: no cover - interpreter shutdown
        pass


def check(status: int) -> None:
    if status != MXMOE_GG_OK:
        msg = lib().mxmoe_gg_last_error().decode(errors="replace")
        raise GGError(status, msg)


def variant_count() -> int:
    return lib().mxmoe_gg_variant_count()


GENERAL_QCFGS = ("fp16", "w8a8_g-1_sym", "w4a4_g-1_sym")


def production_variants(qcfg: str | None = "general") -> list[int]:
    """Compiled variants that compute correct results (``abl_*`` are timing ablations) and have a tile
    body for ``qcfg`` (default "general": fp16, w8a8 and w4a4 — the general-purpose kernels; ``None``:
    every one). The small-batch ``wo3_*`` kernel has fp16, w8a8, w4a4 and weight-only bodies (not
    w4a4_g128, E4M3 or bf16), so it is in the "general" set too."""
    vs = [int(ln.split()[0]) for ln in list_variants() if not ln.split()[1].startswith("abl_")]
    if qcfg is None:
        return vs
    need = GENERAL_QCFGS if qcfg == "general" else (qcfg,)
    return [v for v in vs if all(variant_supports(v, q) for q in need)]


def plan_tiles(problems, variant: int):
    """Host tile table of a plan (mxmoe_gg_plan_tiles; no device needed): (tiles [slots, 8] int32
    with columns prob/m0/n0/cls/ks0/ks1/slab/grp in blockIdx order, rows: table row -> the caller's
    problem index)."""
    import numpy as np

    P = len(problems)
    arr = (GGProblemC * P)(*problems)
    n = ctypes.c_int(0)
    check(lib().mxmoe_gg_plan_tiles(arr, P, variant, None, None, ctypes.byref(n)))
    tiles = np.zeros((n.value, 8), dtype=np.int32)
    rows = np.full(P, -1, dtype=np.int32)
    check(lib().mxmoe_gg_plan_tiles(arr, P, variant, tiles.ctypes.data, rows.ctypes.data, ctypes.byref(n)))
    return tiles, rows


def default_variant() -> int:
    return lib().mxmoe_gg_default_variant()


def list_variants() -> list[str]:
    buf = ctypes.create_string_buffer(1 << 16)
    n = lib().mxmoe_gg_list_variants(buf, len(buf))
    if n < 0:
        check(-n)
    return [ln for ln in buf.value.decode().splitlines() if ln]


def variant_supports(variant: int, qcfg: str) -> bool:
    """Whether a compiled variant has a tile body for ``qcfg`` (weight-only strategies are listed by
    their base name, e.g. ``w4a16``)."""
    from .tile_config import variant_key

    if variant == VARIANT_AUTO:
        return True
    line = list_variants()[variant]
    return f" {variant_key(qcfg)}=TileConfig(" in line


def variant_caps(variant: int) -> int:
    """Capability bits (CAP_*) of a compiled variant (mxmoe_gg_variant_caps): e.g. whether it has the
    fused SiLU epilogue."""
    out = ctypes.c_uint32()
    check(lib().mxmoe_gg_variant_caps(variant, ctypes.byref(out)))
    return out.value


def variant_tile(variant: int, a_bits: int, w_bits: int) -> dict:
    v = [ctypes.c_int32() for _ in range(4)]
    check(lib().mxmoe_gg_variant_tile(variant, a_bits, w_bits, *[ctypes.byref(x) for x in v]))
    return {"BM": v[0].value, "BN": v[1].value, "BK_bytes": v[2].value, "threads": v[3].value}


def repack_weightonly(ref_words, N: int, K: int, w_bits: int):
    """Reference weight-only packed words (numpy uint16 [N*w_bits/16, K], host) -> the kernel's
    uint8 [N, K*w_bits/8] layout (mxmoe_gg_repack_weightonly)."""
    import numpy as np

    src = np.ascontiguousarray(ref_words, dtype=np.uint16)
    out = np.empty((N, K * w_bits // 8), dtype=np.uint8)
    check(lib().mxmoe_gg_repack_weightonly(src.ctypes.data, N, K, w_bits, out.ctypes.data))
    return out


def pack_f6_host(codes, K: int):
    """Packed int4 rows (numpy uint8 [rows, K/2], pack_wxax) -> fp6 images (uint8 [rows,
    f6_row_bytes(K)]) on the host (mxmoe_gg_pack_f6_host; lab library: MXMOE_GG_LIB)."""
    import numpy as np

    src = np.ascontiguousarray(codes, dtype=np.uint8)
    rows = src.shape[0]
    out = np.empty((rows, f6_row_bytes(K)), dtype=np.uint8)
    check(lib().mxmoe_gg_pack_f6_host(src.ctypes.data, rows, K, 0, out.ctypes.data, 0))
    return out


def pack_f6(codes, K: int, out=None, stream=None):
    """Packed int4 rows (uint8 device tensor [rows, K/2]) -> fp6 images on the device
    (mxmoe_gg_pack_f6, asynchronous on ``stream`` / torch's current stream; lab library)."""
    import torch

    if codes.dtype not in (torch.uint8, torch.int8) or codes.dim() != 2 or codes.shape[1] * 2 < K:
        raise ValueError("pack_f6: codes must be a uint8 [rows, >= K/2] tensor")
    rows = codes.shape[0]
    if out is None:
        out = torch.empty((rows, f6_row_bytes(K)), dtype=torch.uint8, device=codes.device)
    s = stream if stream is not None else torch.cuda.current_stream(codes.device)
    check(lib().mxmoe_gg_pack_f6(ctypes.c_void_p(codes.data_ptr()), rows, K, codes.stride(0) // 2,
                                 ctypes.c_void_p(out.data_ptr()), out.stride(0) // 2, ctypes.c_void_p(s.cuda_stream)))
    return out


def resolve_variant(problems, problem_count: int, variant: int = VARIANT_AUTO) -> int:
    """The concrete variant AUTO (or an index) resolves to for a ctypes array of GGProblemC (host only)."""
    out = ctypes.c_int()
    check(lib().mxmoe_gg_resolve_variant(problems, problem_count, variant, ctypes.byref(out)))
    return out.value


def workspace_size(problems, problem_count: int, variant: int) -> int:
    """Workspace bytes for a ctypes array of GGProblemC (plan table + pointers + tile table)."""
    n = ctypes.c_size_t()
    check(lib().mxmoe_gg_workspace_size(problems, problem_count, variant, ctypes.byref(n)))
    return n.value
