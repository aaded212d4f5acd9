"""The product path never imports the oracle (only tests/, smoke() and
bench.py's cpu_baseline leg may), and fails loudly without the HIP library."""
import ast
import glob
import os
import subprocess
import sys

from conftest import ROOT


def _oracle_imports(tree):
    out = []
    for node in ast.walk(tree):
        if isinstance(node, ast.Import):
            out += [(node, a.name) for a in node.names if a.name.split(".")[0] == "oracle"]
        elif isinstance(node, ast.ImportFrom) and (node.module or "").split(".")[0] == "oracle":
            out.append((node, node.module))
    return out


def test_package_never_imports_oracle():
    for path in glob.glob(os.path.join(ROOT, "feddct_amd", "**", "*.py"), recursive=True):
        tree = ast.parse(open(path).read())
        assert not _oracle_imports(tree), path


def test_bench_uses_oracle_only_in_cpu_baseline():
    tree = ast.parse(open(os.path.join(ROOT, "bench.py")).read())
    allowed = set()
    for fn in ast.walk(tree):
        if isinstance(fn, ast.FunctionDef) and fn.name == "run_cpu_baseline":
            allowed |= {id(n) for n in ast.walk(fn)}
    for node, name in _oracle_imports(tree):
        assert id(node) in allowed, f"bench.py imports {name} outside the cpu_baseline leg"


def test_missing_library_fails_loudly(tmp_path):
    """Copy the package without libfedagg.so: importing the binding raises."""
    import shutil
    dst = tmp_path / "feddct_amd"
    shutil.copytree(os.path.join(ROOT, "feddct_amd"), dst,
                    ignore=shutil.ignore_patterns("*.so", "__pycache__"))
    code = "import feddct_amd._lib"
    r = subprocess.run([sys.executable, "-c", code], cwd=tmp_path, capture_output=True, text=True)
    assert r.returncode != 0 and "no CPU fallback" in r.stderr
