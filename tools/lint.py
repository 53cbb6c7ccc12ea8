#!/usr/bin/env python3
"""Minimal static checks (the image has no ruff/flake8): syntax, unused imports, line length,
tabs, trailing whitespace, and bare ``except:``. Exit status 1 on any finding."""
import ast
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DIRS = ["igaming_platform_amd", "tests", "tools"]
FILES = ["bench.py", "__graft_entry__.py"]
MAX = 130


def py_files():
    for d in DIRS:
        for dp, _, fs in os.walk(os.path.join(ROOT, d)):
            if "probe" in dp:  # one-off hardware probes, not product code
                continue
            for f in fs:
                if f.endswith(".py"):
                    yield os.path.join(dp, f)
    for f in FILES:
        yield os.path.join(ROOT, f)


def unused_imports(tree: ast.Module, src: str):
    imported = {}
    for node in ast.walk(tree):
        if isinstance(node, (ast.Import, ast.ImportFrom)):
            if isinstance(node, ast.ImportFrom) and node.module == "__future__":
                continue
            for a in node.names:
                name = (a.asname or a.name).split(".")[0]
                imported.setdefault(name, node.lineno)
    used = {n.id for n in ast.walk(tree) if isinstance(n, ast.Name)}
    used |= {n.value.id for n in ast.walk(tree) if isinstance(n, ast.Attribute) and isinstance(n.value, ast.Name)}
    exported = set()
    for node in ast.walk(tree):
        if isinstance(node, ast.Assign) and any(isinstance(t, ast.Name) and t.id == "__all__" for t in node.targets):
            exported |= {e.value for e in node.value.elts if isinstance(e, ast.Constant)}
    for name, line in imported.items():
        if name not in used and name not in exported and f"{name}" not in src.split("# noqa")[0][-1:]:
            yield line, f"unused import {name!r}"


def main() -> int:
    bad = 0
    for path in py_files():
        rel = os.path.relpath(path, ROOT)
        src = open(path, encoding="utf-8").read()
        try:
            tree = ast.parse(src, rel)
        except SyntaxError as e:
            print(f"{rel}:{e.lineno}: syntax error: {e.msg}")
            bad += 1
            continue
        lines = src.splitlines()
        for i, ln in enumerate(lines, 1):
            if len(ln) > MAX and "http" not in ln:
                print(f"{rel}:{i}: line too long ({len(ln)} > {MAX})")
                bad += 1
            if "\t" in ln:
                print(f"{rel}:{i}: tab character")
                bad += 1
            if ln.rstrip() != ln:
                print(f"{rel}:{i}: trailing whitespace")
                bad += 1
        for node in ast.walk(tree):
            if isinstance(node, ast.ExceptHandler) and node.type is None:
                print(f"{rel}:{node.lineno}: bare except")
                bad += 1
        if not rel.endswith("__init__.py"):
            for line, msg in unused_imports(tree, src):
                if "noqa" not in lines[line - 1]:
                    print(f"{rel}:{line}: {msg}")
                    bad += 1
    print(f"lint: {bad} finding(s)")
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
