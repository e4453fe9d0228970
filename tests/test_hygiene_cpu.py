"""The oracle is test infrastructure: only tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg may import it; the product package never does."""
import ast
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _imports_oracle(node):
    for n in ast.walk(node):
        if isinstance(n, ast.Import) and any(a.name.split(".")[0] == "oracle" for a in n.names):
            return True
        if isinstance(n, ast.ImportFrom) and (n.module or "").split(".")[0] == "oracle":
            return True
    return False


def test_package_never_imports_oracle():
    bad = []
    for d, _, files in os.walk(os.path.join(ROOT, "tmrnet_amd")):
        for f in files:
            if f.endswith(".py"):
                p = os.path.join(d, f)
                if _imports_oracle(ast.parse(open(p).read())):
                    bad.append(os.path.relpath(p, ROOT))
    assert not bad, bad


def test_bench_imports_oracle_only_in_cpu_baseline():
    tree = ast.parse(open(os.path.join(ROOT, "bench.py")).read())
    allowed = {"cpu_baseline"}
    for node in tree.body:
        if isinstance(node, ast.FunctionDef) and node.name in allowed:
            continue
        assert not _imports_oracle(node), getattr(node, "name", type(node).__name__)


def test_bench_rejects_rank_count_mismatch():
    """--gpus N under a launcher with another WORLD_SIZE must fail, not measure silently."""
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    p = subprocess.run([sys.executable, "bench.py", "--gpus", "8"], cwd=ROOT, env=env,
                       capture_output=True, text=True, timeout=120)
    assert p.returncode == 2, (p.returncode, p.stderr[-2000:])
    assert "WORLD_SIZE" in p.stderr
