"""__graft_entry__ (CPU): smoke() runs only on a GPU box, so check here that every helper it imports from
the test utilities exists (the driver calls smoke() at round end)."""
import ast
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_smoke_imports_resolve():
    src = open(os.path.join(ROOT, "__graft_entry__.py")).read()
    fn = next(n for n in ast.parse(src).body if isinstance(n, ast.FunctionDef) and n.name == "smoke")
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    sys.path.insert(0, os.path.join(ROOT, "threestudio-3dgs_amd"))
    import importlib

    checked = 0
    for node in ast.walk(fn):
        if isinstance(node, ast.ImportFrom) and node.module in ("gsr_testutil",):
            mod = importlib.import_module(node.module)
            for alias in node.names:
                assert hasattr(mod, alias.name), f"smoke() imports missing {node.module}.{alias.name}"
                checked += 1
    assert checked >= 5
