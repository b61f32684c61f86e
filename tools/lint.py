"""Blocking lint for the Python tree (CI's lint step; needs nothing beyond the standard library).

Checks, per file:
  * it compiles (syntax);
  * unused imports (an imported name never referenced in the module; ``__init__.py`` re-exports,
    ``__all__`` members and lines marked ``# noqa`` are exempt);
  * a function / class defined twice in the same scope (the first one is dead);
  * comparisons to None / True / False with ``==`` / ``!=``;
  * bare ``except:``;
  * lines longer than 128 characters (the reference's flake8 sets 120, `Server/.flake8:1-4`).

    python tools/lint.py [paths...]        # exit status 1 on any finding
"""
from __future__ import annotations

import ast
import os
import sys
from typing import Iterable, List

MAX_LINE = 128     # (the reference's flake8 allows 120; this tree's wrapped lines run to 128)
DEFAULT_PATHS = ("fed_tgan_amd", "tests", "tools", "dtds", "bench.py", "__graft_entry__.py", "similarity_analysis.py",
                 "utility_analysis.py", "csrc/build.py")


def _py_files(paths: Iterable[str]) -> List[str]:
    out = []
    for p in paths:
        if os.path.isfile(p) and p.endswith(".py"):
            out.append(p)
        elif os.path.isdir(p):
            for root, dirs, files in os.walk(p):
                dirs[:] = [d for d in dirs if d not in ("__pycache__", "golden", "build")]
                out += [os.path.join(root, f) for f in sorted(files) if f.endswith(".py")]
    return sorted(out)


class _Names(ast.NodeVisitor):
    def __init__(self):
        self.used = set()

    def visit_Name(self, node):
        self.used.add(node.id)

    def visit_Attribute(self, node):
        base = node
        while isinstance(base, ast.Attribute):
            base = base.value
        if isinstance(base, ast.Name):
            self.used.add(base.id)
        self.generic_visit(node)


def _string_names(tree) -> set:
    """Names mentioned in string annotations / __all__ (counted as uses)."""
    out = set()
    for node in ast.walk(tree):
        if isinstance(node, ast.Constant) and isinstance(node.value, str) and node.value.isidentifier():
            out.add(node.value)
        if isinstance(node, ast.Constant) and isinstance(node.value, str):
            for tok in node.value.replace("[", " ").replace("]", " ").replace(",", " ").replace(".", " ").split():
                if tok.isidentifier():
                    out.add(tok)
    return out


def lint_file(path: str) -> List[str]:
    src = open(path, encoding="utf-8").read()
    lines = src.splitlines()
    errs = []
    try:
        tree = ast.parse(src, path)
    except SyntaxError as e:
        return [f"{path}:{e.lineno}: syntax error: {e.msg}"]
    for i, line in enumerate(lines, 1):
        if len(line) > MAX_LINE and "noqa" not in line and "http" not in line:
            errs.append(f"{path}:{i}: line too long ({len(line)} > {MAX_LINE})")
    noqa = {i for i, line in enumerate(lines, 1) if "# noqa" in line}
    # unused imports (module level and function level: a name bound by import and never read anywhere)
    if os.path.basename(path) != "__init__.py":
        nv = _Names()
        nv.visit(tree)
        used = nv.used | _string_names(tree)
        for node in ast.walk(tree):
            if isinstance(node, (ast.Import, ast.ImportFrom)):
                if isinstance(node, ast.ImportFrom) and node.module == "__future__":
                    continue
                if node.lineno in noqa or getattr(node, "end_lineno", node.lineno) in noqa:
                    continue
                for a in node.names:
                    if a.name == "*":
                        continue
                    bound = a.asname or a.name.split(".")[0]
                    if bound not in used:
                        errs.append(f"{path}:{node.lineno}: '{a.name}' imported but unused")
    # redefinitions in one scope
    for scope in [tree] + [n for n in ast.walk(tree) if isinstance(n, (ast.ClassDef, ast.FunctionDef,
                                                                       ast.AsyncFunctionDef))]:
        seen = {}
        for st in getattr(scope, "body", []):
            if isinstance(st, (ast.FunctionDef, ast.AsyncFunctionDef, ast.ClassDef)):
                decos = [d for d in st.decorator_list]
                overload = any((isinstance(d, ast.Attribute) and d.attr in ("setter", "getter", "deleter", "register"))
                               or (isinstance(d, ast.Name) and d.id == "overload") for d in decos)
                if st.name in seen and not overload and st.lineno not in noqa:
                    errs.append(f"{path}:{st.lineno}: redefinition of '{st.name}' from line {seen[st.name]}")
                seen[st.name] = st.lineno
    for node in ast.walk(tree):
        if isinstance(node, ast.Compare) and node.lineno not in noqa:
            for op, comp in zip(node.ops, node.comparators):
                if isinstance(op, (ast.Eq, ast.NotEq)) and isinstance(comp, ast.Constant) and \
                        (comp.value is None or comp.value is True or comp.value is False):
                    errs.append(f"{path}:{node.lineno}: comparison to {comp.value} with ==/!= (use 'is')")
        if isinstance(node, ast.ExceptHandler) and node.type is None and node.lineno not in noqa:
            errs.append(f"{path}:{node.lineno}: bare 'except:'")
    return errs


def main(argv=None) -> int:
    argv = sys.argv[1:] if argv is None else argv
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    paths = argv or [os.path.join(root, p) for p in DEFAULT_PATHS]
    errs = []
    files = _py_files(paths)
    for f in files:
        errs += lint_file(f)
    for e in errs:
        print(os.path.relpath(e, root) if e.startswith(root) else e)
    print(f"lint: {len(files)} files, {len(errs)} finding(s)", file=sys.stderr)
    return 1 if errs else 0


if __name__ == "__main__":
    sys.exit(main())
