"""bench.py --gpus N (CPU): the launch decision made before any GPU call, and the child launcher
command. n_gpus in the JSON line is WORLD_SIZE, so --gpus N either runs N ranks or refuses."""
from __future__ import annotations

import subprocess
import sys

import bench


def test_single_gpu_runs_here():
    assert bench.resolve_launch(1, {}, 1) == ("run", "")
    assert bench.resolve_launch(1, {}, 8) == ("run", "")


def test_gpus_n_without_launcher_spawns_ranks():
    assert bench.resolve_launch(8, {}, 8) == ("spawn", "")
    assert bench.resolve_launch(2, {}, 8) == ("spawn", "")


def test_gpus_n_refuses_fewer_gpus_under_rccl():
    act, why = bench.resolve_launch(8, {}, 1)
    assert act == "error" and "visible GPU" in why
    act, _ = bench.resolve_launch(2, {"MXMOE_DIST_BACKEND": "nccl", "MXMOE_DIST_SHARE_GPU": "1"}, 1)
    assert act == "error"  # sharing one GPU is a gloo rehearsal only


def test_gloo_rehearsal_may_share_one_gpu():
    env = {"MXMOE_DIST_BACKEND": "gloo", "MXMOE_DIST_SHARE_GPU": "1"}
    assert bench.resolve_launch(2, env, 1) == ("spawn", "")
    assert bench.resolve_launch(2, {**env, "WORLD_SIZE": "2"}, 1) == ("run", "")
    assert bench.resolve_launch(2, {"MXMOE_DIST_BACKEND": "gloo"}, 1)[0] == "error"  # no opt-in


def test_launcher_world_size_must_equal_gpus():
    assert bench.resolve_launch(8, {"WORLD_SIZE": "8"}, 8) == ("run", "")
    act, why = bench.resolve_launch(8, {"WORLD_SIZE": "1"}, 8)
    assert act == "error" and "WORLD_SIZE=1" in why
    assert bench.resolve_launch(1, {"WORLD_SIZE": "4"}, 8)[0] == "error"
    assert bench.resolve_launch(4, {"WORLD_SIZE": "4"}, 2)[0] == "error"  # ranks would wrap onto GPUs
    assert bench.resolve_launch(0, {}, 8)[0] == "error"


def test_spawn_command_is_torchrun_on_loopback():
    cmd = bench.spawn_ranks(4, ["--gpus", "4", "--steps", "3"])
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nproc-per-node=4" in cmd and "--master-addr=127.0.0.1" in cmd and "--nnodes=1" in cmd
    port = int(next(a for a in cmd if a.startswith("--master-port=")).split("=")[1])
    assert 0 < port < 65536
    assert cmd[-4:] == ["--gpus", "4", "--steps", "3"] and cmd[-5].endswith("bench.py")


def test_bench_refuses_mismatched_world_size_before_gpu_work():
    # WORLD_SIZE=2 with --gpus 3: exits 2 at the launch decision (no GPU, no process group)
    r = subprocess.run([sys.executable, bench.__file__, "--gpus", "3"], env={"WORLD_SIZE": "2", "PATH": "/usr/bin"},
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 2 and "n_gpus must equal --gpus" in r.stderr


def _unresolved_globals(path) -> set:
    """Names a function in ``path`` reads as implicit globals that the module never binds and that are
    not builtins (a pyflakes-style check via symtable: ADVICE r04 found `settle_s` read by
    strong_scaling_step without being its parameter — a NameError swallowed by the extras' except)."""
    import builtins
    import symtable

    top = symtable.symtable(open(path).read(), str(path), "exec")
    bound = {s.get_name() for s in top.get_symbols() if s.is_assigned() or s.is_imported()} | {"__file__", "__name__"}
    bad = set()

    def walk(t):
        for c in t.get_children():
            if c.get_type() in ("function", "lambda"):
                for s in c.get_symbols():
                    if s.is_referenced() and s.is_global() and not s.is_declared_global():
                        n = s.get_name()
                        if n not in bound and not hasattr(builtins, n):
                            bad.add(f"{c.get_name()}:{n}")
            walk(c)

    walk(top)
    return bad


def test_bench_functions_read_no_unbound_names():
    assert _unresolved_globals(bench.__file__) == set()
    import inspect

    assert "settle_s" in inspect.signature(bench.strong_scaling_step).parameters
