"""Static checks (the reference's CI runs mypy + ruff, .gitlab-ci.yml:80-95).

Neither tool is installed in this image, so the checks that matter for this
code base are implemented on the stdlib ``ast``:

* every module of the package imports (no GPU needed);
* every public ``__all__`` name resolves;
* no unused imports outside ``__init__`` re-export modules (ruff F401);
* line length <= 119 (the reference's and our ruff setting);
* no unsafe deserialisation or exec-style process replacement in library code.
"""

from __future__ import annotations

import ast
import importlib
import pkgutil
from pathlib import Path

import pytest

import ddl_amd

ROOT = Path(__file__).resolve().parents[1]
PKG = ROOT / "ddl_amd"
PY_FILES = sorted(p for p in PKG.rglob("*.py") if "__pycache__" not in p.parts) + [
    ROOT / "bench.py", ROOT / "__graft_entry__.py"]


def _modules():
    yield "ddl_amd"
    for m in pkgutil.walk_packages(ddl_amd.__path__, "ddl_amd."):
        yield m.name


@pytest.mark.parametrize("name", sorted(_modules()))
def test_module_imports(name):
    importlib.import_module(name)


def test_public_names_resolve():
    for mod in ("ddl_amd", "ddl_amd.ops", "ddl_amd.parallel", "ddl_amd.models", "ddl_amd.utils"):
        m = importlib.import_module(mod)
        for n in getattr(m, "__all__", []):
            assert getattr(m, n) is not None, f"{mod}.{n}"


def _unused_imports(tree: ast.Module) -> list[str]:
    imported: dict[str, int] = {}
    for node in ast.walk(tree):
        if isinstance(node, ast.Import):
            for a in node.names:
                imported[(a.asname or a.name).split(".")[0]] = node.lineno
        elif isinstance(node, ast.ImportFrom) and node.module != "__future__":
            for a in node.names:
                imported[a.asname or a.name] = node.lineno
    used = {n.id for n in ast.walk(tree) if isinstance(n, ast.Name)}
    used |= {n.value.id for n in ast.walk(tree) if isinstance(n, ast.Attribute) and isinstance(n.value, ast.Name)}
    # names mentioned in string annotations / __all__
    for n in ast.walk(tree):
        if isinstance(n, ast.Constant) and isinstance(n.value, str):
            used |= set(n.value.replace("[", " ").replace("]", " ").replace(",", " ").replace("|", " ").split())
    return [f"{k} (line {v})" for k, v in imported.items() if k not in used]


@pytest.mark.parametrize("path", PY_FILES, ids=lambda p: str(p.relative_to(ROOT)))
def test_lint(path: Path):
    src = path.read_text()
    tree = ast.parse(src)
    problems = []
    if path.name != "__init__.py":
        problems += [f"unused import {u}" for u in _unused_imports(tree)]
    for i, line in enumerate(src.splitlines(), 1):
        if len(line) > 119:
            problems.append(f"line {i} longer than 119")
    for node in ast.walk(tree):
        if isinstance(node, ast.Attribute) and isinstance(node.value, ast.Name):
            if node.value.id == "pickle" and node.attr in ("load", "loads"):
                problems.append(f"pickle.{node.attr} at line {node.lineno}")
            if node.value.id == "os" and node.attr.startswith("exec"):
                problems.append(f"os.{node.attr} at line {node.lineno}")
        if isinstance(node, ast.keyword) and node.arg in ("weights_only", "allow_pickle"):
            bad = node.value.value if isinstance(node.value, ast.Constant) else None
            if (node.arg == "weights_only" and bad is False) or (node.arg == "allow_pickle" and bad is True):
                problems.append(f"{node.arg}={bad} at line {node.value.lineno}")
    assert not problems, f"{path.relative_to(ROOT)}: {problems}"


def test_license_file():
    """The package declares LGPL-2.1-or-later (pyproject, CITATION.cff) and ships the license text."""
    text = (ROOT / "LICENSE").read_text()
    assert text.lstrip().startswith("GNU LESSER GENERAL PUBLIC LICENSE") and "Version 2.1" in text[:200]
    assert "LGPL-2.1" in (ROOT / "pyproject.toml").read_text()
    assert "LGPL-2.1" in (ROOT / "CITATION.cff").read_text()


def _expand_braces(path: str) -> list[str]:
    """``a_{x,y}.json`` -> ``[a_x.json, a_y.json]`` (the docs' shorthand for sibling evidence files)."""
    import re

    m = re.search(r"\{([^{}]*)\}", path)
    if m is None:
        return [path]
    return [q for opt in m.group(1).split(",") for q in _expand_braces(path[:m.start()] + opt + path[m.end():])]


def test_cited_evidence_exists():
    """Every ``profiles/...`` / ``archive/...`` path the README and docs cite as evidence exists in the tree
    (brace and glob shorthand allowed; a bare ``r4_tenth/`` continues a range begun with a full path, so it is
    looked up among the evidence and job directories)."""
    import re

    docs = [ROOT / "README.md", ROOT / "profiles" / "README.md", *sorted((ROOT / "docs").glob("*.md"))]
    pat = re.compile(r"`((?:\.\./)?(?:archive/|profiles/|r[1-6]_)[^`\s]*)`")
    bases = [ROOT, ROOT / "profiles", ROOT / "archive" / "profiles", ROOT / "archive" / "jobs", ROOT / "tools" / "jobs"]
    missing = []
    for doc in docs:
        for m in pat.finditer(doc.read_text()):
            cited = m.group(1).split("::")[0].rstrip(",.)")
            names = [p.rstrip("/") for p in _expand_braces(cited)]
            for base in bases:
                if any(next(base.glob(n.replace("../", "", 1) if base == ROOT else n), None) for n in names):
                    break
            else:
                missing.append(f"{doc.relative_to(ROOT)}: {cited}")
    assert not missing, missing
