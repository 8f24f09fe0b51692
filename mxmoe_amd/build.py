"""Build libmxmoe_gg.so in-tree with hipcc for gfx950 (no JIT cache: the .so travels with the repo)."""
from __future__ import annotations

import os
import subprocess
import sys
from pathlib import Path

PKG = Path(__file__).resolve().parent
ROOT = PKG.parent
CSRC = PKG / "csrc"
LIB = PKG / "lib" / "libmxmoe_gg.so"
# tools-only lab library: the v2 family with the timing ablations and mainloop experiments
# (-DMXMOE_LAB; tools/kbench.py with MXMOE_GG_LIB=<this>). Never loaded by the product.
LAB_LIB = PKG / "lib" / "libmxmoe_gg_lab.so"
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("MXMOE_OFFLOAD_ARCH", "gfx950")

SOURCES = [CSRC / "gg_api.hip", CSRC / "moe_ops.hip"]
DEPS = SOURCES + [CSRC / "gg_device.h", CSRC / "gg_v2q.h", ROOT / "include" / "mxmoe_gg.h", ROOT / "include" / "mxmoe_moe.h"]

FLAGS = ["-O3", "-std=c++17", "-fPIC", "-shared", f"--offload-arch={ARCH}", "-Wall", "-Wno-unused-function",
         "-I", str(ROOT / "include")]


# the lab build also compiles the lab-only kernels' headers
LAB_DEPS = DEPS + [CSRC / "gg_f6.h"]


def needs_build(lib: Path = LIB) -> bool:
    """True when `lib` is missing or older than any source it is built from (the lab library's
    tests skip on a stale lab build: a binary HEAD does not produce must not pass for HEAD's)."""
    if not lib.exists():
        return True
    t = lib.stat().st_mtime
    return any(p.stat().st_mtime > t for p in (LAB_DEPS if lib == LAB_LIB else DEPS))


def build(force: bool = False, verbose: bool = False, extra: list[str] | None = None, lab: bool = False,
          lab_fast: bool = False) -> Path:
    """lab_fast: the lab library with only the experiments under test (-DMXMOE_LAB_FAST; gg_api.hip)."""
    lab = lab or lab_fast
    out = LAB_LIB if lab else LIB
    if not force and not needs_build(out):
        return out
    out.parent.mkdir(parents=True, exist_ok=True)
    tmp = out.with_suffix(".so.tmp")
    defs = (["-DMXMOE_LAB"] if lab else []) + (["-DMXMOE_LAB_FAST"] if lab_fast else [])
    cmd = [HIPCC, *FLAGS, *defs, *(extra or []), "-o", str(tmp), *map(str, SOURCES)]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True)
    os.replace(tmp, out)
    return out


REF_HARNESS_SRC = [ROOT / "tests" / "cpp" / "ref_harness_call.cpp", ROOT / "tests" / "cpp" / "layout_check.cpp"]
REF_HARNESS = ROOT / "tests" / "cpp" / "bin" / "ref_harness_call"


def build_ref_harness(force: bool = False, verbose: bool = False) -> Path:
    """The reference-side C++ caller of groupgemm_mxmoe (tests/cpp): test
    infrastructure, linked against the product library (rpath to mxmoe_amd/lib)."""
    deps = REF_HARNESS_SRC + [ROOT / "include" / "mxmoe_gg.h", LIB]
    if not force and REF_HARNESS.exists() and all(p.stat().st_mtime <= REF_HARNESS.stat().st_mtime for p in deps):
        return REF_HARNESS
    REF_HARNESS.parent.mkdir(parents=True, exist_ok=True)
    cmd = [HIPCC, "-O2", "-std=c++17", f"--offload-arch={ARCH}", "-Wall", "-I", str(ROOT / "include"),
           "-o", str(REF_HARNESS), *map(str, REF_HARNESS_SRC), "-L", str(LIB.parent), "-lmxmoe_gg",
           "-Wl,-rpath,$ORIGIN/../../../mxmoe_amd/lib"]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True)
    return REF_HARNESS


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True, lab="--lab" in sys.argv, lab_fast="--lab-fast" in sys.argv))
