#!/usr/bin/env python3
"""Rewrite ``DistributedDataLoader(..., out_dtype=..., seed=..., prefetch_depth=...)`` calls to the option
records (``output=OutputSpec(...)``, ``order=OrderSpec(...)``, ``staging=StagingSpec(...)``).

Usage: ``python tools/migrate_specs.py FILE...`` (in place). Only calls that pass at least one flat keyword
of ``ddl_amd.specs.LEGACY`` are touched; positional arguments and the other keywords keep their source text.
A call that already passes one of the records is left alone (merge by hand). The records are referenced as
``ddl_amd.<Spec>``; ``import ddl_amd`` is added when the module lacks it.
"""

from __future__ import annotations

import ast
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from ddl_amd.specs import LEGACY  # noqa: E402

SPEC = {"output": "OutputSpec", "staging": "StagingSpec", "order": "OrderSpec"}


def _offset(lines: list[str], lineno: int, col: int) -> int:
    return sum(len(x) for x in lines[: lineno - 1]) + col


def migrate(src: str) -> tuple[str, int]:
    tree = ast.parse(src)
    lines = src.splitlines(keepends=True)
    edits = []
    for node in ast.walk(tree):
        if not isinstance(node, ast.Call):
            continue
        f = node.func
        name = f.attr if isinstance(f, ast.Attribute) else f.id if isinstance(f, ast.Name) else None
        if name != "DistributedDataLoader":
            continue
        kws = [k for k in node.keywords if k.arg in LEGACY]
        if not kws or any(k.arg in SPEC for k in node.keywords):
            continue
        seg = lambda n: ast.get_source_segment(src, n)  # noqa: E731
        parts = [seg(a) for a in node.args]
        groups: dict[str, list[str]] = {"output": [], "staging": [], "order": []}
        for k in node.keywords:
            if k.arg in LEGACY:
                rec, field = LEGACY[k.arg]
                groups[rec].append(f"{field}={seg(k.value)}")
            elif k.arg is None:
                parts.append(f"**{seg(k.value)}")
            else:
                parts.append(f"{k.arg}={seg(k.value)}")
        for rec in ("output", "staging", "order"):
            if groups[rec]:
                parts.append(f"{rec}=ddl_amd.{SPEC[rec]}({', '.join(groups[rec])})")
        line_text = lines[node.lineno - 1]
        head = f"{seg(node.func)}("
        col = node.col_offset + len(head)  # hanging indent aligned with the opening parenthesis
        if col > 60 or any("\n" in p for p in parts):
            indent = len(line_text) - len(line_text.lstrip()) + 4
            head, col = head + "\n" + " " * indent, indent
        out, cur = [], col
        for i, p in enumerate(parts):
            piece = p + (")" if i == len(parts) - 1 else ",")
            if out and out[-1] != "\n" and cur + 1 + len(piece.split("\n")[0]) > 119:
                out.append("\n" + " " * col)
                cur = col
            elif out:
                out.append(" ")
                cur += 1
            out.append(piece)
            cur = (cur + len(piece)) if "\n" not in piece else len(piece.rsplit("\n", 1)[1])
        new = head + "".join(out)
        start = _offset(lines, node.lineno, node.col_offset)
        end = _offset(lines, node.end_lineno, node.end_col_offset)
        edits.append((start, end, new))
    for start, end, new in sorted(edits, reverse=True):
        src = src[:start] + new + src[end:]
    if edits and not any(isinstance(n, ast.Import) and any(a.name == "ddl_amd" and a.asname is None
                                                          for a in n.names) for n in ast.walk(tree)):
        # top-level "import ddl_amd" after the last __future__ / docstring block
        out, done = [], False
        for ln in src.splitlines(keepends=True):
            if not done and (ln.startswith("import ") or ln.startswith("from ")) and "__future__" not in ln:
                out.append("import ddl_amd\n")
                done = True
            out.append(ln)
        src = "".join(out)
    return src, len(edits)


def main(paths: list[str]) -> int:
    for p in paths:
        with open(p) as f:
            src = f.read()
        new, n = migrate(src)
        if n:
            compile(new, p, "exec")
            with open(p, "w") as f:
                f.write(new)
            print(f"{p}: {n} call(s)")
    return 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
