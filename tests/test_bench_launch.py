"""bench.py's own N > 1 launch: `python bench.py --gpus N` started WITHOUT
torchrun spawns N child ranks (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* set by the parent), which
meet at the TCP rendezvous, share the shared-segment name and the RCCL id, and rank 0's JSON line is
relayed.  --dry-run stops before anything loads libmgicp.so, so this runs on the CPU."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("n", [2, 4])
def test_bench_spawns_its_own_ranks(n):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(n), "--dry-run"],
                         capture_output=True, text=True, timeout=120, env=env, cwd=ROOT)
    assert out.returncode == 0, out.stderr
    lines = [ln for ln in out.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1  # only rank 0 prints
    rec = json.loads(lines[0])
    assert rec["dry_run"] and rec["n_gpus"] == n and rec["ranks_joined"] == n and rec["uid_ok"]
    assert rec["local_rank"] == 0 and rec["shm_name"].startswith("/mgicp_")


def test_bench_launch_never_loads_the_engine_in_the_parent():
    """The parent of the spawned ranks must not load libmgicp.so (HIP) -- it only spawns and waits."""
    import ast

    src = open(os.path.join(ROOT, "bench.py")).read()
    tree = ast.parse(src)
    fn = next(f for f in tree.body if isinstance(f, ast.FunctionDef) and f.name == "launch_ranks")
    names = {n.id for n in ast.walk(fn) if isinstance(n, ast.Name)} | \
            {n.attr for n in ast.walk(fn) if isinstance(n, ast.Attribute)}
    assert not names & {"GICPEngine", "_lib", "load", "execv", "execve", "execvp"}
    main = next(f for f in tree.body if isinstance(f, ast.FunctionDef) and f.name == "main")
    first = main.body[:3]  # args, then the launch branch before any engine import
    assert any(isinstance(s, ast.If) and "launch_ranks" in ast.dump(s) for s in first)
